// Minimum-norm least squares for the symmetric Newton systems: the reference's
//   np.linalg.lstsq(H, rhs, rcond=None)
// (NewtonSolver.py:212-227 np_lstsq, :334-341 the Cholesky-failure backup (Q9);
//  NewtonSolverInfeasibleStart.py:279-316 np_lstsq block elimination, :692-724 the diagonal class).
//
// NumPy's lstsq is LAPACK gelsd: singular values s_i <= rcond * s_max are treated as zero, with
// rcond = eps * max(M, N) when rcond is None.  Every matrix the reference hands to lstsq on this
// path is symmetric (H, and S = A H^+ A^T), so its singular values are |lambda_i| and its singular
// vectors are eigenvectors:
//   x = sum_{|lambda_i| > eps n max|lambda|} v_i (v_i^T b) / lambda_i
// which is the gelsd solution up to rounding (the same minimum-norm vector whenever H is
// singular, where an LU solve returns a huge or non-finite step instead).
//
// The eigendecomposition is a hand-written parallel cyclic Jacobi method (no vendor library):
// every round rotates n/2 disjoint index pairs (p, q) at once -- the round-robin "circle"
// ordering visits every pair once per sweep of n-1 rounds -- with the rotation that zeroes A_pq
// (Golub & Van Loan, sym.schur2), applied two-sided to A (each thread owns a 2 x 2 block of A, so
// the update is in place) and to the columns of V.  Sweeps repeat until no off-diagonal entry is
// rotated: |A_pq| <= eps sqrt|A_pp A_qq| (relative), or |A_pq| <= eps ||A||_F / n (absolute:
// the off-diagonal rest then moves an eigenvalue by at most eps ||A||_F, the backward error of
// gelsd itself).  The absolute bound is needed on rank-deficient H: in the null-space block
// A_pp, A_qq and A_pq are all rounding noise of the large rotations, the relative test keeps
// rotating that noise forever (a numpy restatement at n = 1025, rank 700 never stops), and those
// eigenvalues fall below gelsd's cut anyway.  Small systems (n <= JWG_MAX) run the whole iteration in
// ONE workgroup (no launches per round); larger ones one rotation + one update launch per round and
// a 4-byte readback per sweep.  Non-convergence within JMAX_SWEEPS sets *info_dev = 1 (the host
// raises LinAlgError like numpy's "SVD did not converge"); the word is sticky -- a factorization
// never clears it, so of several eigensolves in one Newton step (the block elimination's H and S)
// a failed one cannot be overwritten by a later converged one.
// Right-hand sides use the engine's row-major convention: B is n x nrhs, element (i, j) at
// B[i * ldb + j].
#include <hip/hip_runtime.h>

#include <atomic>
#include <cfloat>
#include <cmath>
#include <vector>

#include "ipm_common.h"

namespace ipm {

constexpr int JWG_MAX = 256;       // single-workgroup path up to this n
constexpr int JMAX_SWEEPS = 60;

// pair i of round r in the circle ordering of nn (even) players: player 0 fixed, the others rotate
__device__ __forceinline__ void circle_pair(int nn, int r, int i, int& a, int& b) {
  const int m = nn - 1;
  a = (i == 0) ? 0 : ((i - 1 + r) % m) + 1;
  b = ((nn - 2 - i + r) % m) + 1;
}

// rotation (c, s) zeroing A_pq (p < q): J = [[c, s], [-s, c]] on rows / columns (p, q)
__device__ __forceinline__ bool jacobi_rot(double app, double aqq, double apq, double tiny, double& c, double& s) {
  const double ap = fabs(apq);
  if (!(ap > DBL_EPSILON * sqrt(fabs(app) * fabs(aqq))) || !(ap > tiny)) {
    c = 1.0;
    s = 0.0;
    return false;
  }
  const double tau = (aqq - app) / (2.0 * apq);
  const double t = (tau >= 0.0 ? 1.0 : -1.0) / (fabs(tau) + sqrt(1.0 + tau * tau));
  c = 1.0 / sqrt(1.0 + t * t);
  s = t * c;
  return true;
}

// pair encoding: p | (q << 16), q = JSINGLE when the pair is an odd n's last index with the dummy
// player -- a single index p that no rotation touches, but whose entries in the rotated rows and
// columns of the OTHER pairs still turn with them
constexpr int JSINGLE = 0xFFFF;
__device__ __forceinline__ int jpack(int p, int q, int n) { return p | ((q < n ? q : JSINGLE) << 16); }

// the block (rows of pair P, columns of pair Q) of A <- J^T A J, in place: 2 x 2 for two real pairs,
// 2 x 1 / 1 x 2 when one side is a single index (identity rotation on that side), nothing for two
// singles
__device__ __forceinline__ void jacobi_block(double* A, int64_t lda, int pp, double c1, double s1, int pq, double c2,
                                             double s2, bool diag) {
  const int p1 = pp & 0xFFFF, q1 = (pp >> 16) & 0xFFFF, p2 = pq & 0xFFFF, q2 = (pq >> 16) & 0xFFFF;
  const bool r2 = q1 != JSINGLE, k2 = q2 != JSINGLE;
  if (r2 && k2) {
    double* a11 = A + (int64_t)p2 * lda + p1;   // (p1, p2)
    double* a12 = A + (int64_t)q2 * lda + p1;   // (p1, q2)
    double* a21 = A + (int64_t)p2 * lda + q1;   // (q1, p2)
    double* a22 = A + (int64_t)q2 * lda + q1;   // (q1, q2)
    const double x11 = *a11, x12 = *a12, x21 = *a21, x22 = *a22;
    // rows: r_p = c r_p - s r_q, r_q = s r_p + c r_q
    const double y11 = c1 * x11 - s1 * x21, y12 = c1 * x12 - s1 * x22;
    const double y21 = s1 * x11 + c1 * x21, y22 = s1 * x12 + c1 * x22;
    // columns: likewise with the column pair's rotation
    double z11 = c2 * y11 - s2 * y12, z12 = s2 * y11 + c2 * y12;
    double z21 = c2 * y21 - s2 * y22, z22 = s2 * y21 + c2 * y22;
    if (diag) {   // the rotated pair itself: symmetric, off-diagonal zero by construction
      z12 = z21 = 0.0;
    }
    *a11 = z11;
    *a12 = z12;
    *a21 = z21;
    *a22 = z22;
  } else if (r2) {   // column p2 alone: rows (p1, q1) turn
    double* a11 = A + (int64_t)p2 * lda + p1;
    double* a21 = A + (int64_t)p2 * lda + q1;
    const double x11 = *a11, x21 = *a21;
    *a11 = c1 * x11 - s1 * x21;
    *a21 = s1 * x11 + c1 * x21;
  } else if (k2) {   // row p1 alone: columns (p2, q2) turn
    double* a11 = A + (int64_t)p2 * lda + p1;
    double* a12 = A + (int64_t)q2 * lda + p1;
    const double x11 = *a11, x12 = *a12;
    *a11 = c2 * x11 - s2 * x12;
    *a12 = s2 * x11 + c2 * x12;
  }
}

__device__ __forceinline__ void jacobi_vcols(double* V, int64_t n, int p, int q, double c, double s, int64_t k) {
  double* vp = V + (int64_t)p * n;
  double* vq = V + (int64_t)q * n;
  const double a = vp[k], b = vq[k];
  vp[k] = c * a - s * b;
  vq[k] = s * a + c * b;
}

// ||A||_F^2 -> *out (one workgroup)
__global__ __launch_bounds__(256) void k_frob2(int64_t n, const double* __restrict__ A, int64_t lda, double* out) {
  __shared__ double red[256];
  double acc = 0.0;
  for (int64_t e = threadIdx.x; e < n * n; e += 256) {
    const double v = A[(e / n) * lda + (e % n)];
    acc = fma(v, v, acc);
  }
  red[threadIdx.x] = acc;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) *out = red[0];
}

__global__ void k_eye(int64_t n, double* V) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < n * n) V[e] = (e / n == e % n) ? 1.0 : 0.0;
}

// whole Jacobi iteration in one workgroup (n <= JWG_MAX): A, V in global memory (L2-resident)
__global__ __launch_bounds__(1024) void k_jacobi_wg(int n, double* A, int64_t lda, double* V, const double* frob2,
                                                    int* info) {
  __shared__ int spart[JWG_MAX + 1];
  __shared__ double sc[JWG_MAX + 1], ss[JWG_MAX + 1];
  __shared__ int srot;
  const int nn = n + (n & 1), half = nn / 2, tid = threadIdx.x;
  const double tiny = DBL_EPSILON * sqrt(*frob2) / (double)n;
  int sweep = 0;
  for (; sweep < JMAX_SWEEPS; ++sweep) {
    if (tid == 0) srot = 0;
    __syncthreads();
    for (int r = 0; r < nn - 1; ++r) {
      for (int i = tid; i < half; i += 1024) {
        int a, b;
        circle_pair(nn, r, i, a, b);
        const int p = min(a, b), q = max(a, b);
        double c = 1.0, s = 0.0;
        if (q < n && jacobi_rot(A[(int64_t)p * lda + p], A[(int64_t)q * lda + q], A[(int64_t)q * lda + p], tiny, c, s))
          atomicAdd(&srot, 1);
        spart[i] = jpack(p, q, n);
        sc[i] = c;
        ss[i] = s;
      }
      __syncthreads();
      // A blocks (pair P, pair Q) and V column pairs
      for (int e = tid; e < half * half; e += 1024) {
        const int P = e / half, Q = e % half;
        const int pp = spart[P], pq = spart[Q];
        if (sc[P] == 1.0 && ss[P] == 0.0 && sc[Q] == 1.0 && ss[Q] == 0.0) continue;
        jacobi_block(A, lda, pp, sc[P], ss[P], pq, sc[Q], ss[Q], P == Q);
      }
      for (int e = tid; e < half * n; e += 1024) {
        const int P = e / n, k = e % n;
        const int pp = spart[P];
        if (sc[P] == 1.0 && ss[P] == 0.0) continue;   // (singles always: identity)
        jacobi_vcols(V, n, pp & 0xFFFF, pp >> 16, sc[P], ss[P], k);
      }
      __syncthreads();
    }
    if (srot == 0) break;
    __syncthreads();
  }
  if (tid == 0 && sweep >= JMAX_SWEEPS) *info = 1;   // sticky: never cleared here
}

// large n: one round = rotations (k_jacobi_rot) + the two-sided update (k_jacobi_upd)
__global__ void k_jacobi_rot(int n, int r, const double* __restrict__ A, int64_t lda, const double* frob2,
                             int* __restrict__ part, double* __restrict__ cs, int* __restrict__ nrot) {
  const int nn = n + (n & 1), half = nn / 2;
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= half) return;
  const double tiny = DBL_EPSILON * sqrt(*frob2) / (double)n;
  int a, b;
  circle_pair(nn, r, i, a, b);
  const int p = min(a, b), q = max(a, b);
  double c = 1.0, s = 0.0;
  if (q < n && jacobi_rot(A[(int64_t)p * lda + p], A[(int64_t)q * lda + q], A[(int64_t)q * lda + p], tiny, c, s))
    atomicAdd(nrot, 1);
  part[i] = jpack(p, q, n);
  cs[2 * i] = c;
  cs[2 * i + 1] = s;
}

__global__ void k_jacobi_upd(int n, double* A, int64_t lda, double* V, const int* __restrict__ part,
                             const double* __restrict__ cs) {
  const int nn = n + (n & 1), half = nn / 2;
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nA = (int64_t)half * half;
  if (e < nA) {
    const int P = (int)(e % half), Q = (int)(e / half);   // consecutive threads: consecutive row pairs
    const int pp = part[P], pq = part[Q];
    const double c1 = cs[2 * P], s1 = cs[2 * P + 1], c2 = cs[2 * Q], s2 = cs[2 * Q + 1];
    if (c1 == 1.0 && s1 == 0.0 && c2 == 1.0 && s2 == 0.0) return;
    jacobi_block(A, lda, pp, c1, s1, pq, c2, s2, P == Q);
  } else if (e < nA + (int64_t)half * n) {
    const int64_t f = e - nA;
    const int P = (int)(f / n);
    const int64_t k = f % n;
    const int pp = part[P];
    if (cs[2 * P] == 1.0 && cs[2 * P + 1] == 0.0) return;   // (singles always: identity)
    jacobi_vcols(V, n, pp & 0xFFFF, pp >> 16, cs[2 * P], cs[2 * P + 1], k);
  }
}

// eigenvalues (diagonal of the rotated A) -> pseudo-inverse weights f_i = 1/lambda_i if
// |lambda_i| > eps * n * max|lambda| else 0 (gelsd's rcond=None rule); V -> A (eigenvectors in place)
__global__ __launch_bounds__(256) void k_jacobi_finish(int64_t n, double* A, int64_t lda, const double* __restrict__ V,
                                                       double* __restrict__ f) {
  __shared__ double red[256];
  double m = 0.0;
  for (int64_t i = threadIdx.x; i < n; i += 256) m = fmax(m, fabs(A[i * lda + i]));
  red[threadIdx.x] = m;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] = fmax(red[threadIdx.x], red[threadIdx.x + w]);
    __syncthreads();
  }
  const double cut = DBL_EPSILON * (double)n * red[0];
  for (int64_t i = threadIdx.x; i < n; i += 256) {
    const double l = A[i * lda + i];
    f[i] = (fabs(l) > cut) ? 1.0 / l : 0.0;
  }
  __syncthreads();   // every diagonal read before V overwrites A
  for (int64_t e = threadIdx.x; e < n * n; e += 256) A[(e / n) * lda + (e % n)] = V[e];
}

// T(i, r) = f_i sum_k V(k, i) B(k, r): one wave per (i, r), lanes split k (V column i contiguous)
__global__ __launch_bounds__(256) void k_vtb(int64_t n, int64_t nrhs, const double* __restrict__ V, int64_t ldv,
                                             const double* __restrict__ B, int64_t ldb, const double* __restrict__ f,
                                             double* __restrict__ T) {
  const int64_t w = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (w >= n * nrhs) return;
  const int64_t i = w / nrhs, r = w % nrhs;
  const double* v = V + i * ldv;
  double acc = 0.0;
  for (int64_t k = lane; k < n; k += 64) acc = fma(v[k], B[k * ldb + r], acc);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) acc += __shfl_xor(acc, o, 64);
  if (lane == 0) T[r * n + i] = f[i] * acc;
}

// B(i, r) = sum_k V(i, k) T(k, r): one thread per (i, r); V(i, k) for fixed k is contiguous in i
__global__ __launch_bounds__(256) void k_vt(int64_t n, int64_t nrhs, const double* __restrict__ V, int64_t ldv,
                                            const double* __restrict__ T, double* __restrict__ B, int64_t ldb) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * nrhs) return;
  const int64_t i = e % n, r = e / n;
  const double* t = T + r * n;
  double acc = 0.0;
  for (int64_t k = 0; k < n; ++k) acc = fma(V[k * ldv + i], t[k], acc);
  B[i * ldb + r] = acc;
}

void lstsq_release(void* rb) { (void)rb; }

static std::atomic<int> g_fail_call{-1};
void set_lstsq_fail_call(int k) { g_fail_call.store(k); }
__global__ void k_set_flag(int* p) { *p = 1; }

// ws: f (n) | frob2 + counters (64) | V (n^2) | rotation pairs (n) + (c, s) (2n) | T (n * nrhs)
int64_t lstsq_ws_doubles(int64_t n, int64_t nrhs) {
  return n + 64 + n * n + 3 * (n + 2) + std::max<int64_t>(nrhs, 1) * n;
}

// A (full symmetric, column-major, lda) -> eigenvectors V in place; ws[0:n] -> pseudo-inverse
// weights f.  *info_dev = 0, or 1 when Jacobi did not converge within JMAX_SWEEPS sweeps.
// Returns 0, or -1 on a launch error.
int lstsq_sym_factor(void** rb, hipStream_t st, int64_t n, double* A, int64_t lda, double* ws, int* info_dev) {
  (void)rb;
  if (n <= 0) return 0;
  if (n >= (1 << 15)) return -1;   // pair packing (16-bit indices)
  double* f = ws;
  double* frob2 = ws + n;
  int* nrot = reinterpret_cast<int*>(ws + n + 8);
  double* V = ws + n + 64;
  int* part = reinterpret_cast<int*>(V + n * n);
  double* cs = V + n * n + (n + 2);
  hipLaunchKernelGGL(k_frob2, dim3(1), dim3(256), 0, st, n, A, lda, frob2);
  hipLaunchKernelGGL(k_eye, dim3((unsigned)((n * n + 255) / 256)), dim3(256), 0, st, n, V);
  if (n <= JWG_MAX) {
    hipLaunchKernelGGL(k_jacobi_wg, dim3(1), dim3(1024), 0, st, (int)n, A, lda, V, frob2, info_dev);
  } else {
    const int nn = (int)(n + (n & 1)), half = nn / 2;
    const int64_t upd = (int64_t)half * half + (int64_t)half * n;
    int sweep = 0;
    for (; sweep < JMAX_SWEEPS; ++sweep) {
      hipMemsetAsync(nrot, 0, sizeof(int), st);
      for (int r = 0; r < nn - 1; ++r) {
        hipLaunchKernelGGL(k_jacobi_rot, dim3((half + 255) / 256), dim3(256), 0, st, (int)n, r, A, lda, frob2, part,
                           cs, nrot);
        hipLaunchKernelGGL(k_jacobi_upd, dim3((unsigned)((upd + 255) / 256)), dim3(256), 0, st, (int)n, A, lda, V,
                           part, cs);
      }
      int h = 0;
      if (hipMemcpyAsync(&h, nrot, sizeof(int), hipMemcpyDeviceToHost, st) != hipSuccess ||
          hipStreamSynchronize(st) != hipSuccess)
        return -1;
      if (h == 0) break;
    }
    if (sweep >= JMAX_SWEEPS) hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(1), 0, st, info_dev);   // sticky
  }
  // debug knob: this call reports non-convergence
  if (g_fail_call.load() >= 0 && g_fail_call.fetch_sub(1) == 0)
    hipLaunchKernelGGL(k_set_flag, dim3(1), dim3(1), 0, st, info_dev);
  hipLaunchKernelGGL(k_jacobi_finish, dim3(1), dim3(256), 0, st, n, A, lda, V, f);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

// B (row-major n x nrhs, ldb) <- V diag(f) V^T B, with V, f from lstsq_sym_factor (same ws).
int lstsq_sym_apply(void** rb, hipStream_t st, int64_t n, int64_t nrhs, const double* V, int64_t ldv, double* B,
                    int64_t ldb, double* ws) {
  (void)rb;
  if (n <= 0 || nrhs <= 0) return 0;
  const double* f = ws;
  double* T = ws + n + 64 + n * n + 3 * (n + 2);
  const int64_t waves = n * nrhs;
  hipLaunchKernelGGL(k_vtb, dim3((unsigned)((waves + 3) / 4)), dim3(256), 0, st, n, nrhs, V, ldv, B, ldb, f, T);
  hipLaunchKernelGGL(k_vt, dim3((unsigned)((n * nrhs + 255) / 256)), dim3(256), 0, st, n, nrhs, V, ldv, T, B, ldb);
  return hipGetLastError() == hipSuccess ? 0 : -1;
}

}  // namespace ipm
