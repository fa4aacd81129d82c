// Batched ADMM Lasso + C ABI: the MI355X restatement of the reference's
// LassoSolver (LassoSolver.py:17-337, chunked form :339-485).
//
//   min_x 1/(2m) ||A x - b||^2 + reg ||x||_1   for S problems at once (columns of b / entries of reg)
//
// Setup (once): Q = (diag(m rho) + A^T A)^-1 by the fp64-MFMA GEMM, the blocked Cholesky and the
// multi-RHS triangular solves of this library (LassoSolver.py:157-189); bA = Q (A^T b).
// Iteration (LassoSolver.py:240-252), ONE launch per iteration:
//   x = bA + Qs (u - alpha)          Qs = -m rho Q, an n x n x S fp64 MFMA product
//   alpha = prox(x + u, reg / rho)   soft threshold, row 0 unpenalised with a bias column
//   u = u + x - alpha
// fused: each workgroup owns a 32 (rows) x 32 (problems) tile of x, its four waves split the
// k = 0..n-1 sum (interleaved 4-row slabs, operands straight from HBM/L2 into MFMA registers) and
// fold their partial tiles through LDS in a fixed order; the epilogue applies prox + dual update to
// the tile, writes x, alpha, u and the next iteration's W = u - alpha (ping-pong buffer: every tile
// reads all of W), and -- on check iterations -- per-tile partial sums of ||x - alpha||^2,
// ||rho (alpha - alpha_prev)||^2, ||alpha||^2, ||u||^2 reduced in a fixed order by a second launch.
// The stopping test reads four doubles back every `check_stop` iterations (LassoSolver.py:270-289).
//
// Layout: every (n x S) matrix is row-major with leading dimension lds (element (i, s) at i lds + s),
// so 16 lanes of an MFMA column read/write 16 consecutive problems of one row.
// Roofline: per iteration 8 n^2 bytes of Qs (HBM; L2/MALL-resident below ~n = 4096) and 2 n^2 S
// flops; MFMA-bound for S >~ 40 problems, HBM-bound below.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "../../include/ipm355.h"
#include "ipm_common.h"
#include "ipm_handle.h"
#include "ipm_mfma.h"

using namespace ipm;

namespace {

constexpr int LT = 32;   // tile: 32 rows x 32 problems

struct AdmmStep {
  int64_t n = 0, S = 0, lds = 0, ldq = 0, ldba = 0;
  const double* Qs = nullptr;   // k-major: row k holds Qs(i, k) for i = 0..n-1 (= (-m rho Q)^T)
  const double* bA = nullptr;
  const double* eta = nullptr;
  double* x = nullptr;
  double* alpha = nullptr;
  double* u = nullptr;
  double* partial = nullptr;    // 4 doubles per tile (check iterations)
  double* kpart = nullptr;      // K-split partial tiles: (tile * ks + z) * LT * LT
  unsigned* kcnt = nullptr;     // K-split arrivals per tile (the last one finishes the tile, resets it)
  double rho = 0.0;
  int ba_bcast = 0, eta_bcast = 0, positive = 0, add_bias = 0, dual_form = 0;
  int qs_blocked = 0;           // Qs tile-blocked (ipm_lasso_block_qs): tile y's k rows contiguous
};

template <bool CHECK, int U = 4>
__global__ __launch_bounds__(256) void k_admm_step(AdmmStep a, const double* __restrict__ W, double* __restrict__ Wn) {
  __shared__ double red[4][LT * (LT + 1)];
  __shared__ double bred[16];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, fr = lane & 15, fk = lane >> 4;
  const int64_t s0 = (int64_t)blockIdx.x * LT, i0 = (int64_t)blockIdx.y * LT;
  const int64_t n = a.n, S = a.S, ldq = a.ldq, lds = a.lds;
  bool iin[2], sin_[2];
#pragma unroll
  for (int t = 0; t < 2; ++t) {
    iin[t] = i0 + 16 * t + fr < n;
    sin_[t] = s0 + 16 * t + fr < S;
  }
  // k row stride of Qs: the tile-blocked copy streams one contiguous span per workgroup (each k
  // row of the plain layout gives this tile only 256 bytes: DRAM page hits are rare)
  const int64_t qst = a.qs_blocked ? LT : ldq;
  const double* qp = a.qs_blocked ? a.Qs + (int64_t)blockIdx.y * n * LT + fr : a.Qs + i0 + fr;
  const double* wp = W + s0 + fr;
  // K split over gridDim.z workgroups (z-th chunk of 16-row multiples)
  const int KS = gridDim.z, z = blockIdx.z;
  const int64_t kchunk = ((n + 16 * KS - 1) / (16 * KS)) * 16;
  const int64_t kbeg = z * kchunk, kend = min(n, kbeg + kchunk);
  dbl4 acc[2][2];
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q) acc[p][q] = dbl4{0.0, 0.0, 0.0, 0.0};
  // wave wv takes the 4-row slabs kb = 4 wv + 16 j; lane row k = kb + fk.  Four slabs per pass:
  // 16 independent loads in flight before the 16 MFMAs that consume them.  (Issuing the next pass's
  // loads before this pass's MFMAs -- register double buffering -- measured slower: 47.6 -> 53.4 us
  // at n = 4097, S = 30, profiles/r3_lasso_pipelined_kernel_stats.csv.)
  for (int64_t kb = kbeg + 4 * wv; kb < kend; kb += 16 * U) {
    double av[U][2], bv[U][2];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t k = kb + 16 * u + fk;
      const bool kin = k < kend;
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        av[u][t] = (kin && iin[t]) ? qp[k * qst + 16 * t] : 0.0;
        bv[u][t] = (kin && sin_[t]) ? wp[k * lds + 16 * t] : 0.0;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int p = 0; p < 2; ++p)
#pragma unroll
        for (int q = 0; q < 2; ++q) acc[p][q] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[u][p], bv[u][q], acc[p][q], 0, 0, 0);
  }
  // lane holds (row 16 p + fk + 4 r, problem 16 q + fr) of the tile (f64 MFMA output map)
#pragma unroll
  for (int p = 0; p < 2; ++p)
#pragma unroll
    for (int q = 0; q < 2; ++q)
#pragma unroll
      for (int r = 0; r < 4; ++r) red[wv][(16 * p + fk + 4 * r) * (LT + 1) + 16 * q + fr] = acc[p][q][r];
  __syncthreads();
  double qv[4];
#pragma unroll
  for (int e4 = 0; e4 < 4; ++e4) {
    const int e = tid + 256 * e4, o = (e >> 5) * (LT + 1) + (e & 31);
    qv[e4] = ((red[0][o] + red[1][o]) + red[2][o]) + red[3][o];
  }
  if (KS > 1) {
    // hand the partial tile over; the last of the KS workgroups of this tile sums all of them in
    // split order (deterministic) and runs the epilogue
    const int64_t tile = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    double* mine = a.kpart + (tile * KS + z) * (LT * LT);
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) st_sc1(&mine[tid + 256 * e4], qv[e4]);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __shared__ int last;
    if (tid == 0)
      last = __hip_atomic_fetch_add(&a.kcnt[tile], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(KS - 1);
    __syncthreads();
    if (!last) return;
#pragma unroll
    for (int e4 = 0; e4 < 4; ++e4) {
      double t = 0.0;
      for (int q = 0; q < KS; ++q) t += ld_sc1(&a.kpart[(tile * KS + q) * (LT * LT) + tid + 256 * e4]);
      qv[e4] = t;
    }
    if (tid == 0) __hip_atomic_store(&a.kcnt[tile], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  double pr = 0.0, pd = 0.0, pa = 0.0, pu = 0.0;
#pragma unroll
  for (int e4 = 0; e4 < 4; ++e4) {
    const int e = tid + 256 * e4, il = e >> 5, sl = e & 31;
    const int64_t i = i0 + il, s = s0 + sl;
    if (i < n && s < S) {
      const double qw = qv[e4];
      const int64_t ix = i * lds + s;
      const double xv = a.bA[i * a.ldba + (a.ba_bcast ? 0 : s)] + qw;   // bA + Qs (u - alpha)
      const double uo = a.u[ix], ao = a.alpha[ix];
      const double eta = a.eta[a.eta_bcast ? 0 : s];
      const double v = xv + uo;
      double an = fmax(v - eta, 0.0);
      if (!a.positive) an -= fmax(-v - eta, 0.0);
      if (a.add_bias && i == 0) an = v;
      const double un = a.dual_form ? uo + (xv - an) : (uo + xv) - an;
      a.x[ix] = xv;
      a.alpha[ix] = an;
      a.u[ix] = un;
      Wn[ix] = un - an;
      if (CHECK) {
        const double r = xv - an, d = a.rho * (an - ao);
        pr = fma(r, r, pr);
        pd = fma(d, d, pd);
        pa = fma(an, an, pa);
        pu = fma(un, un, pu);
      }
    }
  }
  if (CHECK) {
    const int64_t blk = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
    pr = block_sum(pr, bred);
    pd = block_sum(pd, bred);
    pa = block_sum(pa, bred);
    pu = block_sum(pu, bred);
    if (tid == 0) {
      a.partial[4 * blk + 0] = pr;
      a.partial[4 * blk + 1] = pd;
      a.partial[4 * blk + 2] = pa;
      a.partial[4 * blk + 3] = pu;
    }
  }
}

// fixed-order reduction of the per-tile partial sums -> out[0..3]
__global__ __launch_bounds__(256) void k_admm_norms(int64_t nblk, const double* __restrict__ part, double* out) {
  __shared__ double red[16];
  double v[4] = {0.0, 0.0, 0.0, 0.0};
  for (int64_t b = threadIdx.x; b < nblk; b += 256)
#pragma unroll
    for (int c = 0; c < 4; ++c) v[c] += part[4 * b + c];
#pragma unroll
  for (int c = 0; c < 4; ++c) {
    const double t = block_sum(v[c], red);
    if (threadIdx.x == 0) out[c] = t;
  }
}

// loss per problem s (LassoSolver.py:254-268): 1/(2m) sum_r (R(r, s) - b(r, s))^2 + reg_s sum_i g(alpha(i, s)),
// i from 1 with a bias column; g = |.| when absm (the loop's loss: not positive; objective(): positive)
__global__ __launch_bounds__(256) void k_lasso_loss(int64_t m, int64_t n, int64_t S, const double* __restrict__ R,
                                                    int64_t ldr, const double* __restrict__ b, int64_t ldb, int b_bcast,
                                                    const double* __restrict__ al, int64_t lds, const double* reg,
                                                    int reg_bcast, int add_bias, int absm, double* out,
                                                    const int64_t* cols) {
  __shared__ double red[16];
  const int64_t s = blockIdx.x;
  double q = 0.0, l1 = 0.0;
  for (int64_t r = threadIdx.x; r < m; r += 256) {
    const double d = R[r * ldr + s] - b[r * ldb + (b_bcast ? 0 : s)];
    q = fma(d, d, q);
  }
  for (int64_t i = (add_bias ? 1 : 0) + threadIdx.x; i < n; i += 256) {
    const double v = al[i * lds + s];
    l1 += absm ? fabs(v) : v;
  }
  q = block_sum(q, red);
  l1 = block_sum(l1, red);
  if (threadIdx.x == 0) out[cols ? cols[s] : s] = 1.0 / (2.0 * (double)m) * q + reg[reg_bcast ? 0 : s] * l1;
}

// normalize_A (LassoSolver.py:122-123): A /= A.std(axis=0), population std.  One thread per column,
// rows summed in order -- NumPy reduces axis 0 of a C-contiguous array row by row, so mean, variance
// and the quotients are bit-identical to A.std(axis=0).
__global__ __launch_bounds__(256) void k_colstd_scale(int64_t m, int64_t n, double* A, int64_t lda, double* stdv) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  double s = 0.0;
  for (int64_t i = 0; i < m; ++i) s += A[i * lda + j];
  const double mean = s / (double)m;
  double v = 0.0;
  for (int64_t i = 0; i < m; ++i) {
    const double d = A[i * lda + j] - mean;
    v += d * d;
  }
  const double sd = sqrt(v / (double)m);
  if (stdv) stdv[j] = sd;
  for (int64_t i = 0; i < m; ++i) A[i * lda + j] = A[i * lda + j] / sd;
}

// [1 | A] (LassoSolver.py:124-131): out is m x (n + 1), ldo
__global__ void k_bias_hstack(int64_t m, int64_t n, const double* A, int64_t lda, double* out, int64_t ldo) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= m * (n + 1)) return;
  const int64_t i = e / (n + 1), j = e - i * (n + 1);
  out[i * ldo + j] = j == 0 ? 1.0 : A[i * lda + j - 1];
}

__global__ void k_add_diag(int64_t n, double* M, int64_t ld, double v) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) M[i * ld + i] += v;
}

__global__ void k_eye(int64_t n, double* M, int64_t ld) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * n) return;
  const int64_t i = e / n, j = e - i * n;
  M[i * ld + j] = i == j ? 1.0 : 0.0;
}

__global__ void k_scal_rows(int64_t rows, int64_t cols, double* M, int64_t ld, double f1, double f2, int two) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * cols) return;
  const int64_t i = e / cols, j = e - i * cols;
  double v = M[i * ld + j] * f1;
  if (two) v = v * f2;
  M[i * ld + j] = v;
}

// prox (LassoSolver.py:533-558) on an n x S block
__global__ void k_prox(int64_t n, int64_t S, const double* v, int64_t ldv, const double* eta, int eta_bcast,
                       int positive, int add_bias, double* out, int64_t ldo) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * S) return;
  const int64_t i = e / S, s = e - i * S;
  const double x = v[i * ldv + s], et = eta[eta_bcast ? 0 : s];
  double o = fmax(x - et, 0.0);
  if (!positive) o -= fmax(-x - et, 0.0);
  if (add_bias && i == 0) o = x;
  out[i * ldo + s] = o;
}

inline unsigned blocks(int64_t n) { return (unsigned)std::max<int64_t>(1, (n + 255) / 256); }

// row-major out (M x N, ldc) = alpha A^T B + beta out; A: K x M, B: K x N row-major.  As the MFMA
// tile's C(i, j) = sum_k X[k][i] Y[k][j] (column-major C): i <- N (X = B), j <- M (Y = A).
void gemm_tn(hipStream_t st, int64_t M, int64_t N, int64_t K, double alpha, const double* A, int64_t lda,
             const double* B, int64_t ldb, double beta, double* Cm, int64_t ldc) {
  GemmArgs g;
  g.ni = N;
  g.nj = M;
  g.K = K;
  g.X = B;
  g.ldx = ldb;
  g.Y = A;
  g.ldy = lda;
  g.C = Cm;
  g.ldc = ldc;
  g.alpha = alpha;
  g.beta = beta;
  mfma_gemm_launch(st, g);
}

}  // namespace

// ======================================================================= C ABI
extern "C" int ipm_gemm_tn(ipm_handle* h, int64_t M, int64_t N, int64_t K, double alpha, const double* A,
                           int64_t lda, const double* B, int64_t ldb, double beta, double* Cm, int64_t ldc) {
  if (!h || M < 0 || N < 0 || K < 0 || (K > 0 && (lda < M || ldb < N)) || ldc < N) return IPM_INVALID_ARG;
  if (M == 0 || N == 0) return IPM_OK;
  if (K == 0) {
    hipLaunchKernelGGL(k_scal_rows, dim3(blocks(M * N)), dim3(256), 0, h->stream, M, N, Cm, ldc, beta, 1.0, 0);
  } else {
    gemm_tn(h->stream, M, N, K, alpha, A, lda, B, ldb, beta, Cm, ldc);
  }
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_transpose(ipm_handle* h, int64_t rows, int64_t cols, const double* in, int64_t ldi, double* out,
                             int64_t ldo) {
  if (!h || rows < 0 || cols < 0 || ldi < cols || ldo < rows) return IPM_INVALID_ARG;
  if (rows * cols > 0) transpose(h->stream, rows, cols, in, ldi, out, ldo);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_copy(ipm_handle* h, double* dst, const double* src, int64_t n) {
  if (!h || n < 0) return IPM_INVALID_ARG;
  if (n > 0) HIPCHK(h, hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDevice, h->stream));
  return IPM_OK;
}

extern "C" int ipm_lasso_colnorm(ipm_handle* h, int64_t m, int64_t n, double* A, int64_t lda, double* stdv) {
  if (!h || m <= 0 || n < 0 || lda < n) return IPM_INVALID_ARG;
  hipLaunchKernelGGL(k_colstd_scale, dim3(blocks(n)), dim3(256), 0, h->stream, m, n, A, lda, stdv);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_lasso_bias(ipm_handle* h, int64_t m, int64_t n, const double* A, int64_t lda, double* out,
                              int64_t ldo) {
  if (!h || m < 0 || n < 0 || lda < n || ldo < n + 1) return IPM_INVALID_ARG;
  if (m > 0) hipLaunchKernelGGL(k_bias_hstack, dim3(blocks(m * (n + 1))), dim3(256), 0, h->stream, m, n, A, lda, out, ldo);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_lasso_qinv(ipm_handle* h, int64_t m, int64_t n, const double* A, int64_t lda, double rho,
                              double* Q, double* QT, int64_t ldq, int* info) {
  // LassoSolver.py:124-131, 157-189: M = diag(m rho) + A^T A; Q = cho_solve(cho_factor(M), I); QT = Q^T
  if (!h || m < 0 || n <= 0 || lda < n || ldq < n || !Q || !QT) return IPM_INVALID_ARG;
  hipStream_t st = h->stream;
  int rc = ipm_gemm_tn(h, n, n, m, 1.0, A, lda, A, lda, 0.0, QT, ldq);   // A^T A (full, both triangles)
  if (rc != IPM_OK) return rc;
  hipLaunchKernelGGL(k_add_diag, dim3(blocks(n)), dim3(256), 0, st, n, QT, ldq, (double)m * rho);
  HIPCHK(h, hipGetLastError());
  int inf = 0;
  rc = ipm_potrf(h, n, QT, ldq, &inf);   // symmetric: the lower column-major triangle of row-major M
  if (info) *info = inf;
  if (rc != IPM_OK) return rc;
  hipLaunchKernelGGL(k_eye, dim3(blocks(n * n)), dim3(256), 0, st, n, Q, ldq);
  rc = ipm_potrs(h, n, n, QT, ldq, Q, ldq);
  if (rc != IPM_OK) return rc;
  transpose(st, n, n, Q, ldq, QT, ldq);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_lasso_scale(ipm_handle* h, int64_t rows, int64_t cols, double* M, int64_t ld, double f1,
                               double f2, int two) {
  if (!h || rows < 0 || cols < 0 || ld < cols) return IPM_INVALID_ARG;
  if (rows * cols > 0)
    hipLaunchKernelGGL(k_scal_rows, dim3(blocks(rows * cols)), dim3(256), 0, h->stream, rows, cols, M, ld, f1, f2, two);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_lasso_prox(ipm_handle* h, int64_t n, int64_t S, const double* v, int64_t ldv, const double* eta,
                              int eta_bcast, int positive, int add_bias, double* out, int64_t ldo) {
  if (!h || n < 0 || S < 0 || ldv < S || ldo < S) return IPM_INVALID_ARG;
  if (n * S > 0)
    hipLaunchKernelGGL(k_prox, dim3(blocks(n * S)), dim3(256), 0, h->stream, n, S, v, ldv, eta, eta_bcast, positive,
                       add_bias, out, ldo);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_lasso_loss(ipm_handle* h, const ipm_lasso_args* a, int absm, double* out, const int64_t* cols) {
  // R = A alpha (m x S) by the MFMA GEMM (X = alpha, Y = A^T), then one workgroup per problem
  if (!h || !a || !a->AT || !a->R || !a->b || !a->reg) return IPM_INVALID_ARG;
  int rc = ipm_gemm_tn(h, a->m, a->S, a->n, 1.0, a->AT, a->ldat, a->alpha, a->lds, 0.0, a->R, a->S);
  if (rc != IPM_OK) return rc;
  hipLaunchKernelGGL(k_lasso_loss, dim3((unsigned)a->S), dim3(256), 0, h->stream, a->m, a->n, a->S, a->R, a->S,
                     a->b, a->ldb, a->b_bcast, a->alpha, a->lds, a->reg, a->reg_bcast, a->add_bias, absm, out, cols);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

__global__ void k_block_qs(int64_t n, const double* __restrict__ Qs, int64_t ldq, double* __restrict__ Qb) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;   // destination index
  const int64_t nt = (n + LT - 1) / LT;
  if (e >= nt * n * LT) return;
  const int64_t il = e % LT, k = (e / LT) % n, it = e / (LT * n), i = it * LT + il;
  Qb[e] = i < n ? Qs[k * ldq + i] : 0.0;
}

// K split of the iteration GEMM: enough workgroups for the chip (>= ~512), chunks of >= 128 rows
static int admm_ksplit(int64_t n, int64_t S) {
  const int64_t tiles = ((S + LT - 1) / LT) * ((n + LT - 1) / LT);
  // IPM_ADMM_WG: the workgroup target (default 512)
  static const int64_t target = [] { const char* e = getenv("IPM_ADMM_WG"); return e ? atoll(e) : 512LL; }();
  int64_t ks = (target + tiles - 1) / tiles;
  ks = std::min<int64_t>(ks, std::max<int64_t>(n / 128, 1));
  return (int)std::max<int64_t>(1, std::min<int64_t>(ks, 16));
}

// [norm partials: 4 per tile + 8][K-split partial tiles][K-split counters (as doubles)]; must be
// zero-initialised once (the counters reset themselves)
extern "C" int64_t ipm_lasso_partial_doubles(int64_t n, int64_t S) {
  const int64_t tiles = ((S + LT - 1) / LT) * ((n + LT - 1) / LT);
  const int ks = admm_ksplit(n, S);
  return 4 * tiles + 8 + (ks > 1 ? tiles * ks * LT * LT + tiles : 0);
}

extern "C" int64_t ipm_lasso_qb_doubles(int64_t n) { return n > 0 ? ((n + LT - 1) / LT) * LT * n : 0; }

extern "C" int ipm_lasso_block_qs(ipm_handle* h, int64_t n, const double* Qs, int64_t ldq, double* Qb) {
  if (!h || n <= 0 || ldq < n || !Qs || !Qb) return IPM_INVALID_ARG;
  const int64_t tot = ipm_lasso_qb_doubles(n);
  hipLaunchKernelGGL(k_block_qs, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, h->stream, n, Qs, ldq, Qb);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_lasso_admm(ipm_handle* h, const ipm_lasso_args* a, int32_t* iters) {
  // LassoSolver.py:240-337 (__run_admm) / :388-470 (one chunk of __run_admm_chunks)
  if (!h || !a || a->n <= 0 || a->S <= 0 || a->lds < a->S || a->ldq < a->n || a->check_stop <= 0 ||
      a->max_iters < 0 || !a->Qs || !a->bA || !a->eta || !a->x || !a->alpha || !a->u || !a->W0 || !a->W1 ||
      !a->partial)
    return IPM_INVALID_ARG;
  if (a->compute_loss && (!a->gaps || !a->AT || !a->R)) return IPM_INVALID_ARG;
  hipStream_t st = h->stream;
  AdmmStep s;
  s.n = a->n;
  s.S = a->S;
  s.lds = a->lds;
  s.ldq = a->ldq;
  s.ldba = a->ldba;
  s.Qs = a->Qs;
  s.bA = a->bA;
  s.eta = a->eta;
  s.x = a->x;
  s.alpha = a->alpha;
  s.u = a->u;
  s.partial = a->partial;
  s.rho = a->rho;
  s.ba_bcast = a->ba_bcast;
  s.eta_bcast = a->eta_bcast;
  s.positive = a->positive;
  s.add_bias = a->add_bias;
  s.dual_form = a->dual_form;
  s.qs_blocked = a->qs_blocked;
  const int ks = admm_ksplit(a->n, a->S);
  const dim3 grid((unsigned)((a->S + LT - 1) / LT), (unsigned)((a->n + LT - 1) / LT), (unsigned)ks);
  const int64_t nblk = (int64_t)grid.x * grid.y;
  double* norms = a->partial + 4 * nblk;
  if (ks > 1) {
    s.kpart = a->partial + 4 * nblk + 8;
    s.kcnt = reinterpret_cast<unsigned*>(s.kpart + nblk * ks * LT * LT);
  }
  double* W = a->W0;
  double* Wn = a->W1;
  int it = 0;
  for (; it < a->max_iters; ++it) {
    const bool check = it % a->check_stop == a->check_stop - 1;
    // IPM_ADMM_U: 4-row slabs per wave and pass (loads in flight before the MFMAs that use them)
    static const int U = [] { const char* e = getenv("IPM_ADMM_U"); return e ? atoi(e) : 4; }();
    if (U == 8) {
      if (check) hipLaunchKernelGGL((k_admm_step<true, 8>), grid, dim3(256), 0, st, s, W, Wn);
      else hipLaunchKernelGGL((k_admm_step<false, 8>), grid, dim3(256), 0, st, s, W, Wn);
    } else if (U == 16) {
      if (check) hipLaunchKernelGGL((k_admm_step<true, 16>), grid, dim3(256), 0, st, s, W, Wn);
      else hipLaunchKernelGGL((k_admm_step<false, 16>), grid, dim3(256), 0, st, s, W, Wn);
    } else {
      if (check) hipLaunchKernelGGL((k_admm_step<true, 4>), grid, dim3(256), 0, st, s, W, Wn);
      else hipLaunchKernelGGL((k_admm_step<false, 4>), grid, dim3(256), 0, st, s, W, Wn);
    }
    std::swap(W, Wn);
    if (a->compute_loss) {
      const int rc = ipm_lasso_loss(h, a, a->positive ? 0 : 1, a->gaps + (int64_t)it * a->ldg, a->gap_cols);
      if (rc != IPM_OK) return rc;
    }
    if (check) {
      hipLaunchKernelGGL(k_admm_norms, dim3(1), dim3(256), 0, st, nblk, a->partial, norms);
      HIPCHK(h, hipMemcpyAsync(h->hbuf, norms, 4 * sizeof(double), hipMemcpyDeviceToHost, st));
      HIPCHK(h, hipStreamSynchronize(st));
      double v[4];
      std::memcpy(v, h->hbuf, sizeof(v));
      const double r_norm = std::sqrt(v[0]), d_norm = std::sqrt(v[1]);
      const double tol_p = a->stop_multiplier + a->eps_rel * std::sqrt(v[2]);
      const double tol_d = a->stop_multiplier + a->eps_rel * a->rho * std::sqrt(v[3]);
      if (r_norm < tol_p && d_norm < tol_d) break;
    }
  }
  HIPCHK(h, hipGetLastError());
  // the reference leaves `iteration` at the last index; x/alpha/u are current; W == u - alpha
  if (iters) *iters = it < a->max_iters ? it : a->max_iters - 1;
  return IPM_OK;
}
