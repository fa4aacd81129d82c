// Dense fp64 kernels for the interior-point Newton step on MI355X (gfx950).
//
//   gemv_n / gemv_t   slack GEMVs and barrier-gradient GEMV^T   (HBM-bound)
//   syrk_lower        KKT assembly  H = t P + C^T diag(w) C + diag(d)   and the
//                     Cholesky trailing update, on v_mfma_f64_16x16x4_f64
//   potrf_lower       blocked right-looking Cholesky (column-major lower)
//   trsm_lower_*      blocked triangular solves (one launch per block column)
//   getrf / getrs     LU with partial pivoting: the Cholesky-failure fallback
//
// Reference call sites replaced: FunctionManager.py:123, 256-258, 301-306, 801-805
// (cuBLAS gemv/gemm via CuPy); NewtonSolver.py:286-313 (cuSOLVER potrf + 2 trsv);
// NewtonSolverInfeasibleStart.py:398-452 (potrf + trsm with p right-hand sides).
#include <atomic>
#include "ipm_common.h"
#include <cstdio>
#include "ipm_mfma.h"

#include <algorithm>
#include <map>
#include <mutex>
#include <queue>
#include <cmath>
#include <tuple>
#include <vector>
#include <cstdlib>
#include <cstring>

namespace ipm {

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// =====================================================================================
// GEMV (row-major M):  y = alpha * M x + beta * y        one wave per row
// =====================================================================================
template <bool VEC>
__device__ __forceinline__ void gemv_row(int64_t row, int64_t cols, double alpha, const double* __restrict__ M,
                                         int64_t ldm, const double* __restrict__ x, double beta,
                                         double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const double* mr = M + row * ldm;
  double acc0 = 0.0, acc1 = 0.0;
  if (VEC) {
    // four 16-byte loads of the row in flight per lane (one per 64-lane stride), eight partial
    // sums folded in a fixed order: the row streams at HBM rate instead of one load per trip
    const int64_t c2 = cols >> 1;
    const double2* m2 = reinterpret_cast<const double2*>(mr);
    const double2* x2 = reinterpret_cast<const double2*>(x);
    double a[8] = {0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0, 0.0};
    int64_t j = lane;
    typedef double nt2 __attribute__((ext_vector_type(2)));
    // two trips' loads in flight (eight per lane), folded trip by trip: the same partial sums in
    // the same order as one trip at a time (bitwise), twice the bytes in flight per wave
    for (; j + 448 < c2; j += 512) {
      nt2 u[8];
      double2 v[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) u[q] = __builtin_nontemporal_load(reinterpret_cast<const nt2*>(m2 + j + 64 * q));
#pragma unroll
      for (int q = 0; q < 8; ++q) v[q] = x2[j + 64 * q];
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        a[2 * (q & 3)] = fma(u[q].x, v[q].x, a[2 * (q & 3)]);
        a[2 * (q & 3) + 1] = fma(u[q].y, v[q].y, a[2 * (q & 3) + 1]);
      }
    }
    for (; j + 192 < c2; j += 256) {
      nt2 u[4];
      double2 v[4];
#pragma unroll
      for (int q = 0; q < 4; ++q) u[q] = __builtin_nontemporal_load(reinterpret_cast<const nt2*>(m2 + j + 64 * q));
#pragma unroll
      for (int q = 0; q < 4; ++q) v[q] = x2[j + 64 * q];
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        a[2 * q] = fma(u[q].x, v[q].x, a[2 * q]);
        a[2 * q + 1] = fma(u[q].y, v[q].y, a[2 * q + 1]);
      }
    }
    for (; j < c2; j += 64) {
      const double2 u = m2[j], v = x2[j];
      a[0] = fma(u.x, v.x, a[0]);
      a[1] = fma(u.y, v.y, a[1]);
    }
    acc0 = (a[0] + a[2]) + (a[4] + a[6]);
    acc1 = (a[1] + a[3]) + (a[5] + a[7]);
    if ((cols & 1) && lane == 0) acc0 = fma(mr[cols - 1], x[cols - 1], acc0);
  } else {
    for (int64_t j = lane; j < cols; j += 64) acc0 = fma(mr[j], x[j], acc0);
  }
  double s = wave_sum(acc0 + acc1);
  if (lane == 0) y[row] = (beta == 0.0) ? alpha * s : alpha * s + beta * y[row];
}

template <bool VEC>
__global__ __launch_bounds__(256) void k_gemv_n(int64_t rows, int64_t cols, double alpha,
                                                const double* __restrict__ M, int64_t ldm,
                                                const double* __restrict__ x, double beta,
                                                double* __restrict__ y) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  gemv_row<VEC>(row, cols, alpha, M, ldm, x, beta, y);
}

// y1 = M1 x (rows r1) and y2 = M2 x (rows r2) in one launch, each row exactly as k_gemv_n computes
// it (the Newton step's C x and P x: one launch fewer per use)
template <bool VEC>
__global__ __launch_bounds__(256) void k_gemv_n2(int64_t cols, const double* __restrict__ x, int64_t r1,
                                                 const double* __restrict__ M1, int64_t ld1, double* __restrict__ y1,
                                                 int64_t r2, const double* __restrict__ M2, int64_t ld2,
                                                 double* __restrict__ y2) {
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row < r1) gemv_row<VEC>(row, cols, 1.0, M1, ld1, x, 0.0, y1);
  else if (row - r1 < r2) gemv_row<VEC>(row - r1, cols, 1.0, M2, ld2, x, 0.0, y2);
}

static bool gemv_vec(const double* M, int64_t ldm, const double* x) {
  return ((ldm & 1) == 0) && ((((uintptr_t)M) & 15) == 0) && ((((uintptr_t)x) & 15) == 0);
}

void gemv_n2(hipStream_t st, int64_t cols, const double* x, int64_t r1, const double* M1, int64_t ld1, double* y1,
             int64_t r2, const double* M2, int64_t ld2, double* y2) {
  if (r1 <= 0 || r2 <= 0 || gemv_vec(M1, ld1, x) != gemv_vec(M2, ld2, x)) {
    // (mixed alignment: two launches keep each product bitwise what gemv_n gives)
    gemv_n(st, r1, cols, 1.0, M1, ld1, x, 0.0, y1);
    gemv_n(st, r2, cols, 1.0, M2, ld2, x, 0.0, y2);
    return;
  }
  dim3 g(cdiv(r1 + r2, 4)), b(256);
  if (gemv_vec(M1, ld1, x))
    hipLaunchKernelGGL(k_gemv_n2<true>, g, b, 0, st, cols, x, r1, M1, ld1, y1, r2, M2, ld2, y2);
  else
    hipLaunchKernelGGL(k_gemv_n2<false>, g, b, 0, st, cols, x, r1, M1, ld1, y1, r2, M2, ld2, y2);
}

void gemv_n(hipStream_t st, int64_t rows, int64_t cols, double alpha, const double* M, int64_t ldm,
            const double* x, double beta, double* y) {
  if (rows <= 0) return;
  dim3 g(cdiv(rows, 4)), b(256);
  const bool vec = gemv_vec(M, ldm, x);
  if (vec)
    hipLaunchKernelGGL(k_gemv_n<true>, g, b, 0, st, rows, cols, alpha, M, ldm, x, beta, y);
  else
    hipLaunchKernelGGL(k_gemv_n<false>, g, b, 0, st, rows, cols, alpha, M, ldm, x, beta, y);
}

// =====================================================================================
// GEMV^T (row-major M):  y[j] = alpha * sum_i (w[i] x[i]) M[i][j] + beta * y[j]
// stage 1: grid (column blocks of 256, row chunks) -> partials [chunk][cols]
// stage 2: fixed-order sum over chunks (deterministic)
// =====================================================================================
__global__ __launch_bounds__(256) void k_gemv_t_part(int64_t rows, int64_t cols, int64_t rchunk,
                                                     const double* __restrict__ M, int64_t ldm,
                                                     const double* __restrict__ x,
                                                     const double* __restrict__ w,
                                                     double* __restrict__ part) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t r0 = (int64_t)blockIdx.y * rchunk;
  const int64_t r1 = min(rows, r0 + rchunk);
  if (j >= cols) return;
  double acc = 0.0;
  for (int64_t i = r0; i < r1; ++i) {
    double xi = w ? w[i] * x[i] : x[i];
    acc = fma(M[i * ldm + j], xi, acc);
  }
  part[(int64_t)blockIdx.y * cols + j] = acc;
}

__global__ __launch_bounds__(256) void k_gemv_t_fin(int64_t cols, int64_t nchunk, double alpha,
                                                    const double* __restrict__ part, double beta,
                                                    double* __restrict__ y) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= cols) return;
  double s = 0.0;
  int64_t c = 0;
  for (; c + 8 <= nchunk; c += 8) {   // loads batched, sums in chunk order
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = part[(c + q) * cols + j];
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  for (; c < nchunk; ++c) s += part[c * cols + j];
  y[j] = (beta == 0.0) ? alpha * s : alpha * s + beta * y[j];
}

// k_gemv_t_fin (alpha 1, beta 0) with the barrier gradient assembled from its column sum in the
// same thread: ct[j], then g[j] exactly as k_grad_combine forms it
__global__ __launch_bounds__(256) void k_gemv_t_fin_grad(int64_t cols, int64_t nchunk, const double* __restrict__ part,
                                                         double* __restrict__ ct, const double* __restrict__ go,
                                                         const double* __restrict__ blb, const double* __restrict__ bub,
                                                         bool ct_first, double* __restrict__ g) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= cols) return;
  double s = 0.0;
  int64_t c = 0;
  for (; c + 8 <= nchunk; c += 8) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = part[(c + q) * cols + j];
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  for (; c < nchunk; ++c) s += part[c * cols + j];
  const double ctj = 1.0 * s;
  ct[j] = ctj;
  double v;
  if (ct_first) {
    v = go ? go[j] : 0.0;
    v = go ? v + ctj : ctj;
    if (blb) v = v - blb[j];
    if (bub) v = v + bub[j];
  } else {
    v = go ? go[j] : 0.0;
    if (blb) v = v - blb[j];
    if (bub) v = v + bub[j];
    v = v + ctj;
  }
  g[j] = v;
}

static void gemv_t_plan(int64_t rows, int64_t cols, int64_t* rchunk, int64_t* nchunk) {
  int64_t cb = cdiv(cols, 256);
  int64_t want = std::max<int64_t>(1, 2048 / std::max<int64_t>(cb, 1));
  int64_t rc = std::max<int64_t>(16, cdiv(rows, want));
  *rchunk = rc;
  *nchunk = std::max<int64_t>(1, cdiv(rows, rc));
}

int64_t gemv_t_ws_elems(int64_t rows, int64_t cols) {
  int64_t rc, nc;
  gemv_t_plan(rows, cols, &rc, &nc);
  return nc * cols;
}

void gemv_t(hipStream_t st, int64_t rows, int64_t cols, double alpha, const double* M, int64_t ldm,
            const double* x, const double* w, double beta, double* y, double* part,
            int64_t part_elems) {
  if (cols <= 0) return;
  int64_t rc, nc;
  gemv_t_plan(rows, cols, &rc, &nc);
  if (rows <= 0) {
    nc = 0;
  }
  if (nc * cols > part_elems) {  // not enough scratch: one chunk
    rc = std::max<int64_t>(rows, 1);
    nc = rows > 0 ? 1 : 0;
  }
  if (nc > 0) {
    dim3 g(cdiv(cols, 256), nc), b(256);
    hipLaunchKernelGGL(k_gemv_t_part, g, b, 0, st, rows, cols, rc, M, ldm, x, w, part);
  }
  hipLaunchKernelGGL(k_gemv_t_fin, dim3(cdiv(cols, 256)), dim3(256), 0, st, cols, nc, alpha, part,
                     beta, y);
}

void gemv_t_grad(hipStream_t st, int64_t rows, int64_t cols, const double* M, int64_t ldm, const double* x,
                 double* ct, double* part, int64_t part_elems, const double* go, const double* blb,
                 const double* bub, bool ct_first, double* g) {
  if (cols <= 0) return;
  int64_t rc, nc;
  gemv_t_plan(rows, cols, &rc, &nc);
  if (rows <= 0) nc = 0;
  if (nc * cols > part_elems) {
    rc = std::max<int64_t>(rows, 1);
    nc = rows > 0 ? 1 : 0;
  }
  if (nc > 0) {
    dim3 gr(cdiv(cols, 256), nc), b(256);
    hipLaunchKernelGGL(k_gemv_t_part, gr, b, 0, st, rows, cols, rc, M, ldm, x, nullptr, part);
  }
  hipLaunchKernelGGL(k_gemv_t_fin_grad, dim3(cdiv(cols, 256)), dim3(256), 0, st, cols, nc, part, ct, go, blb,
                     bub, ct_first, g);
}

// =====================================================================================
// SYRK / GEMM^T on fp64 MFMA: the tile kernel lives in ipm_mfma.h (k_mfma_gemm).
//   H(i,j) = alpha * sum_k w[k] X[k][i] Y[k][j] + beta*H(i,j) + tP*P[j][i] + [i==j] dvec[i]
//   for the lower triangle i >= j; H column-major (element (i,j) at j*ldh + i).
// =====================================================================================
static int num_cus();
static void syrk_launch(hipStream_t st, int64_t n, int64_t k, double alpha, const double* X, int64_t ldx,
                        const double* Y, int64_t ldy, const double* w, double beta, double* H, int64_t ldh,
                        const SyrkEpi& e, const int* info) {
  if (n <= 0) return;
  GemmArgs a;
  a.ni = a.nj = n;
  a.K = k;
  a.X = X;
  a.ldx = ldx;
  a.Y = Y ? Y : X;
  a.ldy = Y ? ldy : ldx;
  a.w = w;
  a.C = H;
  a.ldc = ldh;
  a.alpha = alpha;
  a.beta = beta;
  a.P = e.P;
  a.ldp = e.ldp;
  a.tP = e.tP;
  a.dvec = e.dvec;
  a.info = info;
  a.tri = 1;
  if (e.split_ws) mfma_gemm_launch_split(st, a, e.split_ws, e.split_cap, 2 * num_cus(), e.flags_zero && !info);
  else mfma_gemm_launch(st, a);
}

void syrk_lower(hipStream_t st, int64_t n, int64_t k, double alpha, const double* X, int64_t ldx,
                const double* Y, int64_t ldy, const double* w, double beta, double* H, int64_t ldh,
                const SyrkEpi& epi) {
  syrk_launch(st, n, k, alpha, X, ldx, Y, ldy, w, beta, H, ldh, epi, nullptr);
}

// C(m x n, col-major) -= A(m x k, col-major) B(n x k, col-major)^T   (Cholesky panel / look-ahead)
static void gemm_nt_sub_launch(hipStream_t st, int64_t m, int64_t n, int64_t k, const double* A,
                               int64_t lda, const double* B, int64_t ldb, double* C, int64_t ldc,
                               const int* info) {
  if (m <= 0 || n <= 0 || k <= 0) return;
  GemmArgs a;
  a.ni = m;
  a.nj = n;
  a.K = k;
  a.X = A;
  a.ldx = lda;
  a.Y = B;
  a.ldy = ldb;
  a.C = C;
  a.ldc = ldc;
  a.info = info;
  a.sub = 1;
  mfma_gemm_launch(st, a);
}

void gemm_nt_sub(hipStream_t st, int64_t m, int64_t n, int64_t k, const double* A, int64_t lda,
                 const double* B, int64_t ldb, double* C, int64_t ldc) {
  gemm_nt_sub_launch(st, m, n, k, A, lda, B, ldb, C, ldc, nullptr);
}

void gemm_kk(hipStream_t st, int64_t ni, int64_t nj, int64_t k, const double* X, int64_t ldx, const double* Y,
             int64_t ldy, double* C, int64_t ldc) {
  if (ni <= 0 || nj <= 0) return;
  GemmArgs a;
  a.ni = ni;
  a.nj = nj;
  a.K = k;
  a.X = X;
  a.ldx = ldx;
  a.Y = Y;
  a.ldy = ldy;
  a.C = C;
  a.ldc = ldc;
  a.alpha = 1.0;
  a.beta = 0.0;
  mfma_gemm_launch(st, a);
}

// =====================================================================================
// Cholesky panel (width nb <= 128) in two launches, no redundant work:
//   k_potrf_diag : ONE workgroup factors the nb x nb diagonal block in LDS (16 x 16 blocks,
//                  left-looking, MFMA block updates), writes L11 in place and the inverses
//                  of its eight 16 x 16 diagonal blocks Dinv_J = L_JJ^-1 to a workspace.
//   k_potrf_trsm : rows below the block, L21 = A21 L11^-T, 64 rows per workgroup, 16 rows
//                  per wave.  Each wave runs the 8-step block forward substitution entirely in
//                  MFMA registers: X_J = (B_J - sum_{P<J} X_P L_JP^T) Dinv_J^T.
// LAPACK potrf failure rule: pivot <= 0 or NaN -> info = global column (1-based), first
// failure wins; every later kernel of the factorisation early-exits on *info != 0.
// f64 MFMA 16x16x4 maps (cdna_hip_programming.md §3): A lane l: A[l&15][l>>4];
// B lane l: B[l>>4][l&15]; D lane l, reg r: D[(l>>4)+4r][l&15].  All tiles are kept
// TRANSPOSED (D[j][i] = T[i][j]): then 16 consecutive lanes hold 16 consecutive rows of a
// column-major tile, and the accumulator registers of one product are directly the B
// operands (k-steps s = r) of the next one -- no shuffles or LDS round trips on the chains.
// =====================================================================================
#ifndef IPM_CH_NB
#define IPM_CH_NB 256
#endif
constexpr int PF_NB = 128;   // panel width
constexpr int PF_RB = 64;    // rows per TRSM workgroup
constexpr int CH_NB = IPM_CH_NB;   // outer block (trailing-update depth)
constexpr int PF_DINV = 8 * 256;  // workspace doubles: the eight Dinv blocks, then the packed L11 (36 blocks)

__device__ __forceinline__ unsigned ld_ctl(unsigned* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// packed lower 16x16-block storage: block (I,J), I >= J, at bidx(I,J)*256, element (r,c) at c*16+r
__device__ __forceinline__ int bidx(int I, int J) { return (I * (I + 1)) / 2 + J; }

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// acc -= xb[lane l of this 16-lane row] * x  (one v_fmac_f64 with a DPP row broadcast of src0;
// gfx90a+ DPP64 supports row_newbcast).  l must fold to a constant.  nop: the first use of a
// freshly written xb carries the s_nop of the DPP read-after-VALU-write hazard in the same asm
// statement (the compiler cannot move the producer between them).
__device__ __forceinline__ void fmac_bcast16(double& acc, double xb, double x, int l, bool nop = false) {
  switch (l) {
    case 0:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:0 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 1:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:1 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 2:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:2 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 3:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 4:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:4 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 5:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 6:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:6 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:6 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 7:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:7 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:7 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 8:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:8 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:8 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 9:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:9 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:9 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 10:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:10 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:10 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 11:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:11 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:11 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 12:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:12 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:12 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 13:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:13 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:13 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 14:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:14 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:14 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
    case 15:
      if (nop) asm volatile("s_nop 1\n\tv_fmac_f64_dpp %0, -%1, %2 row_newbcast:15 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      else asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:15 row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x));
      break;
  }
}

// lane l of this 16-lane row, broadcast to the row (DPP row_newbcast; l must fold to a constant)
__device__ __forceinline__ double bcast16(double x, int l) {
  switch (l) {
#define IPM_BC(k) case k: return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + k, 0xf, 0xf, false);
    IPM_BC(0) IPM_BC(1) IPM_BC(2) IPM_BC(3) IPM_BC(4) IPM_BC(5) IPM_BC(6) IPM_BC(7)
    IPM_BC(8) IPM_BC(9) IPM_BC(10) IPM_BC(11) IPM_BC(12) IPM_BC(13) IPM_BC(14) IPM_BC(15)
#undef IPM_BC
  }
  return 0.0;
}

#if defined(IPM_ROLE_TRACE) && !defined(IPM_STAMPS)
#define IPM_STAMPS 1   // (the role-trace build also stamps the traced launch's P(a) diagonal role)
#endif
#ifdef IPM_STAMPS
// phase stamps of a diagonal role (labs; the role-trace build: the traced launch's P(a) role)
__device__ unsigned long long ipm_stamps[128];
#define STAMP() do { if (stamp_on && tid == 0) ipm_stamps[nst] = __builtin_amdgcn_s_memtime(); ++nst; } while (0)
#define STAMPAT(i) do { if (stamp_on && lane == 0) ipm_stamps[i] = __builtin_amdgcn_s_memtime(); } while (0)
#else
#define STAMP() do {} while (0)
#define STAMPAT(i) do {} while (0)
#endif

// 1/sqrt(x) for the Cholesky pivots (x > 0, normal): v_rsq_f64 plus one third-order correction
//   e = 1 - x y0^2,  y = y0 + y0 e (1/2 + 3/8 e)
// (the OCML sequence without its special-value selects, which only matter for x <= 0, inf,
// denormals: a pivot <= 0 is reported as a failure before its value is used).
__device__ __forceinline__ double rsqrt_pivot(double x) {
  const double y0 = __builtin_amdgcn_rsq(x);
  const double e = fma(-x * y0, y0, 1.0);
  return fma(y0 * e, fma(e, 0.375, 0.5), y0);
}

// Dinv = L^-1 of a 16 x 16 lower block stored column-major at sblk (element (r,c) at c*16 + r),
// rinv[r] = 1 / L_rr.  Lane c < 16 computes column c:
//   X[r][c] = (d_rc - sum_{c<=k<r} L[r][k] X[k][c]) / L_rr ;  written to out (column-major).
__device__ __forceinline__ void tri_inverse16(const double* sblk, const double* rinv, double* out, int lane,
                                              bool sc1) {
  const int c = lane & 15;
  double x[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    double v = (r == c) ? 1.0 : 0.0;
#pragma unroll
    for (int k = 0; k < r; ++k) v = fma(-sblk[k * 16 + r], x[k], v);
    x[r] = (r >= c) ? v * rinv[r] : 0.0;
    // each row stored as soon as it is final: inside the fused factorization these sc1 stores
    // go to a loaded memory system, and the role's end-of-iteration store wait then covers only
    // the last rows instead of all 16 (r5k: the wait was 1.3-2.2K cycles per iteration)
    if (lane < 16) {
      if (sc1) st_sc1(&out[c * 16 + r], x[r]);
      else out[c * 16 + r] = x[r];
    }
  }
}

// Dinv_J computed by the leaf (row-major in LDS, element (r, c) at 16 r + c) -> out, column-major
// (element (r, c) at 16 c + r), one wave
__device__ __forceinline__ void publish_dinv(const double* t, double* out, int lane, bool sc1) {
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int gi = q * 64 + lane;
    const double v = t[(gi & 15) * 16 + (gi >> 4)];
    if (sc1) st_sc1(&out[gi], v);
    else out[gi] = v;
  }
}

// One workgroup, 4 waves.  Chain per 16-column block J: MFMA update of block column J ->
// wave 0 factors L_JJ in registers -> waves 0-1 solve the tiles below by substitution.  The
// inverses Dinv_J the TRSM kernel needs are computed by wave 3 while wave 0 factors the NEXT
// block, i.e. off the chain.
// Diagonal-block role.  pubL != null: the fused panel kernel's producer -- every final 16 x 16
// block of L11 is also stored to pubL (packed, sc1) and Dinv_J to dinv_out (sc1); after the
// barrier that follows each block row's completion, thread 0 raises *progress (sc1).
struct DiagSmem {
  double sD[36 * 256];   // L11 (identity-padded beyond nb)
  double srinv[8 * 16];  // 1 / L_cc per diagonal block
  double sdinv[2 * 256];  // V & 2097152: Dinv_J from the leaf (row-major), double-buffered by J
  int fail;
  int rd1;               // wave 1 holds its copy of leaf J's diagonal rows: J + 1 (see the leaf)
};

// FUSED: inside the one-launch-per-block factorisation (k_potrf_block): the panel was written by
// other workgroups of the same launch (sc1 loads), and failures are also recorded in *failw.
// V (variants, tools/chol_lab.hip): bit 0 -- the leaf waves wait only for the PREVIOUS leaf's
// published stores at the end of an iteration (progress J+1 needs block row J: tiles from leaves
// < J and the diagonal block stored by wave 2 in iteration J+1, never the current leaf's rows);
// bit 1 -- branch-free LDS loads / stores around the leaf (clamped addresses + selects).
#ifndef IPM_STEP1_PAIR
#define IPM_STEP1_PAIR 1
#endif
#ifndef IPM_FOLD_ACC
#define IPM_FOLD_ACC 1
#endif
#ifndef IPM_DIAG_V
// 130: branch-free leaf LDS traffic + look-ahead tiles off wave 3 (tools/chol_lab.hip: 73.0K -> 66.7K
// cycles); + 65536 lean leaf tail, 262144 L11 written back after the last progress word, 524288
// later leaves' tiles published by the free waves, 1048576 wave 3 takes a look-ahead tile while two
// waves run the leaf (r5 stamps, profiles/r5i: time to the role's last progress word 70.1K -> 61.8K);
// + 2097152 Dinv from the leaf sweep (profiles/r5m: in the launch 69.8K -> 57.1K stamped cycles,
// POTRF n = 2048 0.713 -> 0.638 ms, the factor bitwise unchanged)
#define IPM_DIAG_V (130 + 65536 + 262144 + 524288 + 1048576 + 2097152)
#endif
template <bool FUSED = false, int V = 0>
__device__ __forceinline__ void diag_role(int64_t k0, int nb, double* __restrict__ A, int64_t lda,
                                          double* __restrict__ dinv_out, int* __restrict__ info,
                                          double* pubL, unsigned* progress, DiagSmem& sm,
                                          unsigned* failw = nullptr, bool stamp_on = true) {
  (void)stamp_on;
  double* sD = sm.sD;
  double* srinv = sm.srinv;
  int& fail = sm.fail;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;   // 4 waves
  const int fr = lane & 15, fk = lane >> 4;
#ifdef IPM_STAMPS
  int nst = 0;
#endif
#ifndef IPM_DIAG_PRIO
#define IPM_DIAG_PRIO 3
#endif
  // the diagonal chain is the critical path; its CU-mates are trailing-update tiles
  if (FUSED && IPM_DIAG_PRIO > 0) __builtin_amdgcn_s_setprio(IPM_DIAG_PRIO);
  if (tid == 0) fail = 0;
  if (tid == 0) sm.rd1 = 0;
  STAMP();
  const int i0 = 2 * (tid & 63), jb = tid >> 6;
  if (nb == PF_NB && ((lda & 1) == 0) && ((k0 & 1) == 0)) {
    // ---- full panel: the 36 lower blocks go global -> LDS directly (global_load_lds_dwordx4,
    //      one wave instruction = 8 columns x 16 rows of one block = 1 KB, lane-linear in the
    //      column-major block image); all 72 in flight at once, 18 per wave.  Upper parts of the
    //      diagonal blocks arrive as whatever memory holds there: never read (see step 2).
    int cnt = 0;
#pragma unroll
    for (int I = 0; I < 8; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J)
#pragma unroll
        for (int h = 0; h < 2; ++h, ++cnt)
          if ((cnt & 3) == wv) {
            const double* src = A + (k0 + J * 16 + (lane >> 3) + 8 * h) * lda + k0 + I * 16 + 2 * (lane & 7);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)&sD[bidx(I, J) * 256 + h * 128],
                                             16, 0, FUSED ? 16 : 0);   // aux 16 = sc1
          }
    if (!FUSED && *info != 0) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    // ---- partial panel (last one): register path with identity padding beyond nb
    const bool vec = ((lda & 1) == 0) && ((k0 & 1) == 0);
    const int ic0 = min(i0, nb - 1), ic1 = min(i0 + 1, nb - 1);
    const double* base = A + k0 * lda + k0;
    double2 v[32];
    if (!FUSED && vec && i0 + 1 < nb) {
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const int jc = min(jb + 4 * q, nb - 1);
        v[q] = *reinterpret_cast<const double2*>(base + jc * lda + i0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const int jc = min(jb + 4 * q, nb - 1);
        v[q].x = FUSED ? ld_sc1(base + jc * lda + ic0) : base[jc * lda + ic0];
        v[q].y = FUSED ? ld_sc1(base + jc * lda + ic1) : base[jc * lda + ic1];
      }
    }
    if (!FUSED && *info != 0) return;
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int j = jb + 4 * q;
      if ((i0 >> 4) >= (j >> 4)) {
        double2 u;
        u.x = (i0 < j) ? 0.0 : ((i0 < nb && j < nb) ? v[q].x : (i0 == j ? 1.0 : 0.0));
        u.y = (i0 + 1 < j) ? 0.0 : ((i0 + 1 < nb && j < nb) ? v[q].y : (i0 + 1 == j ? 1.0 : 0.0));
        *reinterpret_cast<double2*>(&sD[bidx(i0 >> 4, j >> 4) * 256 + (j & 15) * 16 + (i0 & 15)]) = u;
      }
    }
  }
  __syncthreads();
  STAMP();
  // T_IK -= L_IP L_KP^T on one 16 x 16 tile (transposed MFMA layout, see above)
  auto tile_update = [&](int I, int K, int P) {
    const int cb = bidx(I, K) * 256 + fk * 16 + fr;
    const int ab = bidx(K, P) * 256 + fk * 16 + fr, bb = bidx(I, P) * 256 + fk * 16 + fr;
    dbl4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = sD[cb + 64 * r];
    double av[4], bv[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      av[s4] = -sD[ab + 64 * s4];
      bv[s4] = sD[bb + 64 * s4];
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc, 0, 0, 0);
#pragma unroll
    for (int r = 0; r < 4; ++r) sD[cb + 64 * r] = acc[r];
  };
  // two tiles T_{I1,K}, T_{I2,K} -= L_{I,P} L_KP^T at once: the shared L_KP operand loaded once and
  // the two 4-MFMA chains interleaved (each tile's operations exactly tile_update's)
  auto tile_update2 = [&](int I1, int I2, int K, int P) {
    const int o = fk * 16 + fr;
    const int c1 = bidx(I1, K) * 256 + o, c2 = bidx(I2, K) * 256 + o;
    const int ab = bidx(K, P) * 256 + o, b1 = bidx(I1, P) * 256 + o, b2 = bidx(I2, P) * 256 + o;
    dbl4 x1, x2;
#pragma unroll
    for (int r = 0; r < 4; ++r) { x1[r] = sD[c1 + 64 * r]; x2[r] = sD[c2 + 64 * r]; }
    double av[4], v1[4], v2[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      av[s4] = -sD[ab + 64 * s4];
      v1[s4] = sD[b1 + 64 * s4];
      v2[s4] = sD[b2 + 64 * s4];
    }
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) {
      x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], v1[s4], x1, 0, 0, 0);
      x2 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], v2[s4], x2, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) { sD[c1 + 64 * r] = x1[r]; sD[c2 + 64 * r] = x2[r]; }
  };
  // T_IK -= sum_{P < np} L_IP L_KP^T (two accumulators)
  auto tile_update_n = [&](int I, int K, int np) {
    const int o = fk * 16 + fr, cb = bidx(I, K) * 256 + o;
    dbl4 x0, x1 = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int r = 0; r < 4; ++r) x0[r] = sD[cb + 64 * r];
    for (int P = 0; P < np; ++P) {
      const int ab = bidx(K, P) * 256 + o, bb = bidx(I, P) * 256 + o;
      double av[4], bv[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        av[s4] = -sD[ab + 64 * s4];
        bv[s4] = sD[bb + 64 * s4];
      }
      x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[0], bv[0], x0, 0, 0, 0);
      x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[1], bv[1], x1, 0, 0, 0);
      x0 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[2], bv[2], x0, 0, 0, 0);
      x1 = __builtin_amdgcn_mfma_f64_16x16x4f64(av[3], bv[3], x1, 0, 0, 0);
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) sD[cb + 64 * r] = x0[r] + x1[r];
  };
  // T_{I_t,K} -= sum_{P < np} L_{I_t,P} L_KP^T for up to 3 tiles I_t of ONE block column K at
  // once (mask: which t are present): the L_KP operand is shared, each term's loads are issued
  // before the previous term's MFMAs (two terms in flight), so the LDS latency is paid once per
  // term for all tiles instead of once per term and tile
  auto tile_update_multi = [&](const int* It, unsigned mask, int K, int np) {
    const int o = fk * 16 + fr;
    dbl4 x[3];
#pragma unroll
    for (int t = 0; t < 3; ++t) {
      x[t] = dbl4{0.0, 0.0, 0.0, 0.0};
      if (mask & (1u << t)) {
        const int cb = bidx(It[t], K) * 256 + o;
#pragma unroll
        for (int r = 0; r < 4; ++r) x[t][r] = sD[cb + 64 * r];
      }
    }
    double av[4], bv[3][4];
    auto ld = [&](int P) {
      const int ab = bidx(K, P) * 256 + o;
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) av[s4] = -sD[ab + 64 * s4];
#pragma unroll
      for (int t = 0; t < 3; ++t)
        if (mask & (1u << t)) {
          const int bb = bidx(It[t], P) * 256 + o;
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4) bv[t][s4] = sD[bb + 64 * s4];
        }
    };
    if (np > 0) ld(0);
    for (int P = 0; P < np; ++P) {
      double a2[4], b2[3][4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) {
        a2[s4] = av[s4];
#pragma unroll
        for (int t = 0; t < 3; ++t) b2[t][s4] = bv[t][s4];
      }
      if (P + 1 < np) ld(P + 1);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4)
#pragma unroll
        for (int t = 0; t < 3; ++t)
          if (mask & (1u << t)) x[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(a2[s4], b2[t][s4], x[t], 0, 0, 0);
    }
#pragma unroll
    for (int t = 0; t < 3; ++t)
      if (mask & (1u << t)) {
        const int cb = bidx(It[t], K) * 256 + o;
#pragma unroll
        for (int r = 0; r < 4; ++r) sD[cb + 64 * r] = x[t][r];
      }
  };
  // final block column Jc of L11 -> A (lower part of the diagonal tile; i, j < nb); tiles
  // I = Jc + part, Jc + part + parts, ...
  auto write_back = [&](int Jc, int part, int parts) {
    // lane: rows r2, r2+1 of columns c0 and c0+8 of each tile (16-byte stores when aligned)
    const int r2 = 2 * (lane & 7), c0 = lane >> 3;
    const bool v2 = ((lda & 1) == 0) && ((k0 & 1) == 0);
    for (int I = Jc + part; I < 8; I += parts) {
      const int cb = bidx(I, Jc) * 256;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int c = c0 + 8 * h, i = I * 16 + r2, j = Jc * 16 + c;
        const double2 v = *reinterpret_cast<const double2*>(&sD[cb + c * 16 + r2]);
        double* dst = A + (k0 + j) * lda + k0 + i;
        if (FUSED) {
          // write-through (sc1): with a leading dimension that is not a whole number of 128-byte
          // lines, the line holding the block's last rows also holds the first rows of the row
          // chunk below, which other workgroups of this launch write and read (sc1); a plain store
          // would keep that line, with their rows as they were, in this XCD's L2
          if (j < nb) {
            if (i < nb && (I > Jc || r2 >= c)) st_sc1(dst, v.x);
            if (i + 1 < nb && (I > Jc || r2 + 1 >= c)) st_sc1(dst + 1, v.y);
          }
        } else if (v2 && I > Jc && i + 1 < nb && j < nb) {
          *reinterpret_cast<double2*>(dst) = v;
        } else if (j < nb) {
          if (i < nb && (I > Jc || r2 >= c)) dst[0] = v.x;
          if (i + 1 < nb && (I > Jc || r2 + 1 >= c)) dst[1] = v.y;
        }
      }
    }
  };
  // Left-looking with one block column of look-ahead: term P (block column P of L, final after
  // step 3 of iteration P) reaches block column P+1 in step 1 of iteration P+1 (4 MFMAs per
  // tile; for the diagonal tile that is all the chain waits for); block column J+1 receives
  // terms 0..J-1 during the leaf of iteration J (waves 1-2, off the chain).  A partial panel
  // (the last one) stops after its last 16-column block: beyond nb there is only identity padding.
  const int nJ = (nb + 15) >> 4;
  for (int J = 0; J < nJ; ++J) {
    // ---- 1. term J-1 on block column J: wave 0 the diagonal tile, waves 1-3 the tiles below
    if (J > 0) {
#if IPM_STEP1_PAIR
      // waves 1-3 with two tiles below run them as one interleaved pair
      if (wv > 0 && wv + 3 < 8 - J) tile_update2(J + wv, J + wv + 3, J, J - 1);
      else
#endif
      for (int tI = (wv == 0 ? 0 : wv); tI < 8 - J; tI += (wv == 0 ? 8 : 3)) tile_update(J + tI, J, J - 1);
      __syncthreads();   // the leaf waves read tiles other waves updated
    }
    STAMP();
    // ---- 2. factor the 16 x 16 block (J,J) in registers, lane r = row r (16-lane groups hold
    //      copies), AND solve the tiles below it in the same sweep: lane group g of wave w holds
    //      row r of tile (J+1+4w+g, J).  Right-looking, no lane masks: entries above the diagonal
    //      turn into garbage but are never read -- every broadcast reads lane c2 > c or the pivot
    //      lane.  The pivot chain is minimal: the next pivot is formed from two values read before
    //      this column is scaled, l = A[c+1][c] dv_c, piv' = A[c+1][c+1] - l^2 (bitwise what the
    //      vector update leaves in lane c+1), so dv_c -> dv_{c+1} is mul, fma, rsqrt; scaling and
    //      rank-1 updates (one v_fmac_f64 with a DPP row broadcast of column c each) run beside it.
    //      Wave 1 joins (a redundant copy of the chain) for the tiles wave 0 has no group for.
    const int nbt = 7 - J;                                   // tiles below the diagonal one
    // V & 32768 (one register stream): group 0 of each leaf wave holds the diagonal block's rows,
    // groups 1-3 the rows of three tiles below; the multipliers L[c2][c] come from group 0 through
    // SGPRs (v_readlane), so diagonal and tile rows share ONE v_fma per column pair instead of a
    // DPP fmac on a copy of the diagonal rows plus a second one on the tile rows.  Bitwise the
    // same arithmetic as the two-stream sweep (same fma operands).  Leaf waves: 0, 1 while more
    // than 3 tiles are below, 2 for the seventh (J = 0, when waves 2-3 have no other work).
    constexpr bool ONE = (V & 32768) != 0;
    // V & 2097152 (Dinv from the leaf): the lane group after the last tile (Ib == 8) sweeps the
    // identity rows, X = I L^-T: lane r ends with column r of Dinv = L^-1, by the same fma
    // sequence as tri_inverse16 (operand by operand: starts at d_rc, subtracts L[r][k] x[k] for
    // k = 0, 1, .. in order, scales by the pivot factor) -- bitwise the same inverse, and wave 3 is
    // free.  Needs a second leaf wave at J = 3 (wave 0's four groups hold tiles 4-7).
    constexpr bool DL = (V & 2097152) != 0;
    const bool leafw = ONE ? (wv == 0 || (wv == 1 && nbt > 3) || (wv == 2 && nbt > 6))
                           : ((wv == 0) || (wv == 1 && (nbt > 4 || (DL && nbt == 4))));
    if (ONE && leafw) {
      const int db = bidx(J, J) * 256;
      const int rr = lane & 15, g = lane >> 4;
      const int It = J + 3 * wv + g;                         // g >= 1: this lane group's tile
      const bool tval = g > 0 && It < 8;
      const int src = tval ? bidx(It, J) * 256 : db;         // absent tiles: a harmless diagonal copy
      double row[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) row[c] = sD[src + c * 16 + rr];
      int bad = 0;
      double dvs[16];
      double piv = readlane_d(row[0], 0);
      double dv = rsqrt_pivot(piv);
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (!(piv > 0.0) && bad == 0) bad = c + 1;
        dvs[c] = dv;
        double pivn = 1.0, dvn = 1.0;
        if (c + 1 < 16) {
          const double a1 = readlane_d(row[c], c + 1);
          const double d1 = readlane_d(row[c + 1], c + 1);
          const double l1 = a1 * dv;
          pivn = fma(-l1, l1, d1);
          dvn = rsqrt_pivot(pivn);
        }
        row[c] *= dv;   // diagonal lane c: L_cc; other diagonal lanes: L[r][c]; tile lanes: X[r][c]
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) row[c2] = fma(-readlane_d(row[c], c2), row[c], row[c2]);
        piv = pivn;
        dv = dvn;
      }
      if (tval) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          sD[src + c * 16 + rr] = row[c];
          if (pubL) st_sc1(&pubL[src + c * 16 + rr], row[c]);
        }
      }
      if (wv == 0) {
        double mine = dvs[0];
#pragma unroll
        for (int c = 1; c < 16; ++c) mine = (lane == c) ? dvs[c] : mine;
        if (lane < 16) {
          srinv[J * 16 + lane] = mine;
#pragma unroll
          for (int c = 0; c < 16; ++c) sD[db + c * 16 + rr] = (rr >= c) ? row[c] : 0.0;   // column-major
        }
        if (lane == 0 && bad) fail = J * 16 + bad;
      }
      STAMPAT(32 + J);
    } else if (leafw) {
      const int db = bidx(J, J) * 256;
      const int rr = lane & 15;
      const int Ib = J + 1 + 4 * wv + (lane >> 4);
      const bool bval = Ib < 8;
      const bool idg = DL && Ib == 8;
      const int bb = bidx(bval ? Ib : J, J) * 256;
      double row[16], rowb[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        row[c] = sD[db + c * 16 + rr];
        if (V & 2) rowb[c] = sD[bb + c * 16 + rr];   // bb == db for absent tiles: a harmless copy
        else rowb[c] = bval ? sD[bb + c * 16 + rr] : 0.0;
        if (DL) rowb[c] = idg ? (c == rr ? 1.0 : 0.0) : rowb[c];
      }
      // Wave 0 writes the factored diagonal rows back over db at the end of its sweep, and wave 1
      // (a second leaf wave while more than four tiles are below, J <= 3) reads the unfactored
      // ones from db at the start of its own, with no barrier between: wave 1 says when its copy
      // has landed, and wave 0 waits for that before it overwrites db.  (r6: a trailing tile on
      // the same CU -- LDS and issue contention -- delayed wave 1 past wave 0's sweep in ~2 % of
      // the n = 8193 factorizations: tiles J+5.. and Dinv_3 swept from factored rows, silently
      // wrong; the round-5 sleep beside critical roles had kept that CU free.)
      if (wv == 1) {
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        if (lane == 0) __hip_atomic_store(&sm.rd1, J + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      }
      int bad = 0;
      double dvs[16];
      // V & 65536 (lean tail): the failure test is one sum of the 16 pivot factors dv (NaN for a
      // pivot <= 0 or NaN, so the sum is not < inf), read once after the sweep; the exact first
      // failing column is recovered only on that (rare) path
      double dsum = 0.0;
      auto sweep = [&]() {
      double piv = readlane_d(row[0], 0);
      double dv = rsqrt_pivot(piv);
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (V & 65536) {
          // (the failure test's sum is formed after the sweep, as a tree)
        } else if (!(piv > 0.0) && bad == 0) bad = c + 1;
        dvs[c] = dv;
        double pivn = 1.0, dvn = 1.0;
        if (c + 1 < 16) {
          const double a1 = readlane_d(row[c], c + 1);
          const double d1 = readlane_d(row[c + 1], c + 1);
          const double l1 = a1 * dv;
          pivn = fma(-l1, l1, d1);
          dvn = rsqrt_pivot(pivn);
        }
        row[c] *= dv;                      // lane c: piv * dv = L_cc
        rowb[c] *= dv;                     // X[r][c] of the tile below
        if (V & 16) {
          // the broadcast as a compiler builtin (v_mov_b64 DPP row_newbcast), shared by both row
          // sets; plain fmas the scheduler can place
#pragma unroll
          for (int c2 = c + 1; c2 < 16; ++c2) {
            const double bc = bcast16(row[c], c2);
            row[c2] = fma(-bc, row[c], row[c2]);
            rowb[c2] = fma(-bc, rowb[c], rowb[c2]);
          }
        } else if (V & 64) {
          // tile-below rows: the multiplier L[c2][c] read into SGPRs (v_readlane), plain v_fma
#pragma unroll
          for (int c2 = c + 1; c2 < 16; ++c2) {
            fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
            rowb[c2] = fma(-readlane_d(row[c], c2), rowb[c], rowb[c2]);
          }
        } else if (V & 32) {
          // diag rows: the DPP fmac; tile-below rows: the broadcast once more as a DPP mov + fma
#pragma unroll
          for (int c2 = c + 1; c2 < 16; ++c2) {
            fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
            rowb[c2] = fma(-bcast16(row[c], c2), rowb[c], rowb[c2]);
          }
        } else if (V & 1024) {   // lab timing only: no tile-below rows (wrong factor)
#pragma unroll
          for (int c2 = c + 1; c2 < 16; ++c2) fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
        } else {
#pragma unroll
          for (int c2 = c + 1; c2 < 16; ++c2) {
            fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
            fmac_bcast16(rowb[c2], row[c], rowb[c], c2, false);
          }
        }
        piv = pivn;
        dv = dvn;
      }
      };
      if (V & 8192) {   // lab timing only: the sweep twice (the second one warm), stamp between
        double row0[16], rowb0[16];
#pragma unroll
        for (int c = 0; c < 16; ++c) { row0[c] = row[c]; rowb0[c] = rowb[c]; }
        sweep();
        STAMPAT(16 + J);
#pragma unroll
        for (int c = 0; c < 16; ++c) { row[c] = row0[c]; rowb[c] = rowb0[c]; }
        bad = 0;
        dsum = 0.0;
      }
#ifdef IPM_STAMPS
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");   // (stamped lab builds: the sweep alone)
      STAMPAT(48 + J);
#endif
      sweep();
#ifdef IPM_STAMPS
      STAMPAT(56 + J);
#endif
      if (DL && (bval || idg)) {
        // tile rows to their block; the identity group's Dinv rows -- lane r holds Dinv[c][r] --
        // to sdinv row-major (element (c, r) at 16 c + r): one store stream, no divergence
        double* dst = bval ? &sD[bb] : &sm.sdinv[(J & 1) * 256];
#pragma unroll
        for (int c = 0; c < 16; ++c) dst[c * 16 + rr] = rowb[c];
        if (bval && pubL && !(V & 4096) && !((V & 524288) && J >= 2)) {
#pragma unroll
          for (int c = 0; c < 16; ++c) st_sc1(&pubL[bb + c * 16 + rr], rowb[c]);
        }
      } else if (bval) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          sD[bb + c * 16 + rr] = rowb[c];
          // (4096: lab timing only; 524288: leaves J >= 2 are published from LDS by the free waves
          // in the next iteration)
          if (pubL && !(V & 4096) && !((V & 524288) && J >= 2)) st_sc1(&pubL[bb + c * 16 + rr], rowb[c]);
        }
      }
      if ((V & 65536) && wv == 0) {
        // the diagonal rows as they are (the upper part of a diagonal block is never read: the
        // inverse, the write-back and the row roles use its lower part only) and the 16 pivot
        // factors -- wave-uniform values -- from ONE lane: no per-lane selects.  Not before wave 1
        // (when it sweeps this leaf too) holds its copy of the unfactored rows (above).
        if (nbt > 4 || (DL && nbt == 4)) {
          while (__hip_atomic_load(&sm.rd1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < J + 1)
            __builtin_amdgcn_s_sleep(1);
        }
        if (lane < 16) {
#pragma unroll
          for (int c = 0; c < 16; ++c) sD[db + c * 16 + rr] = row[c];   // column-major
        }
        if (lane == 0 && !DL) {   // (Dinv from the leaf needs no pivot factors in LDS)
#pragma unroll
          for (int c = 0; c < 16; ++c) srinv[J * 16 + c] = dvs[c];
        }
        // the 16 pivot factors summed as a tree (4 dependent adds instead of 16 on the leaf's tail):
        // NaN for any pivot <= 0 or NaN, like the running sum, and nothing else reads it
        {
          double t8[8], t4[4];
#pragma unroll
          for (int c = 0; c < 8; ++c) t8[c] = dvs[2 * c] + dvs[2 * c + 1];
#pragma unroll
          for (int c = 0; c < 4; ++c) t4[c] = t8[2 * c] + t8[2 * c + 1];
          dsum = (t4[0] + t4[1]) + (t4[2] + t4[3]);
        }
        if (!(dsum < __builtin_inf())) {   // a pivot <= 0 or NaN (LAPACK potrf's test), rare
#pragma unroll
          for (int c = 15; c >= 0; --c)
            if (!(dvs[c] > 0.0)) bad = c + 1;
          if (lane == 0) fail = J * 16 + bad;
        }
      } else if (wv == 0) {
        if (V & 2) {
          double mine = dvs[0];
#pragma unroll
          for (int c = 1; c < 16; ++c) mine = (lane == c) ? dvs[c] : mine;
          if (lane < 16) {
            srinv[J * 16 + lane] = mine;
#pragma unroll
            for (int c = 0; c < 16; ++c) sD[db + c * 16 + rr] = (rr >= c) ? row[c] : 0.0;   // column-major
          }
        } else if (lane < 16) {
#pragma unroll
          for (int c = 0; c < 16; ++c)
            if (lane == c) srinv[J * 16 + c] = dvs[c];
#pragma unroll
          for (int c = 0; c < 16; ++c) sD[db + c * 16 + rr] = (rr >= c) ? row[c] : 0.0;   // column-major
        }
        if (lane == 0 && bad) fail = J * 16 + bad;
      }
      STAMPAT(32 + J);
    } else if (J > 0) {
      // the other waves, off the chain: wave 3 inverts the PREVIOUS diagonal block for the row
      // part; wave 2 publishes it and writes block column J-1 back to A; the free waves apply
      // terms 0..J-1 to the tiles of block column J+1 (look-ahead)
      if (DL && wv == 3) {
        publish_dinv(&sm.sdinv[((J - 1) & 1) * 256], dinv_out + (J - 1) * 256, lane, pubL != nullptr);
        STAMPAT(40 + J);
      } else if (wv == 3 && !(V & 8)) {   // (V & 8: lab timing only -- the free waves skip their work)
        tri_inverse16(&sD[bidx(J - 1, J - 1) * 256], &srinv[(J - 1) * 16], dinv_out + (J - 1) * 256, lane,
                      pubL != nullptr);
        STAMPAT(40 + J);
      }
      if (wv == 2 && pubL) {
        const int db = bidx(J - 1, J - 1) * 256;
#pragma unroll
        for (int q = 0; q < 4; ++q) st_sc1(&pubL[db + q * 64 + lane], sD[db + q * 64 + lane]);
      }
      if ((V & 524288) && pubL && J >= 3) {
        // the previous leaf's tiles (I, J-1), I >= J, from LDS to pubL, spread over the free waves:
        // tile (I, J-1) belongs to block row I, released (progress > I) at the end of iteration I
        // >= J at the earliest -- after this iteration's store wait and barrier.  (Leaves 0 and 1
        // publish their own: in iterations 1-2 the free waves have no slack.)
        const int fw0 = (ONE ? nbt > 3 : (nbt > 4 || (DL && nbt == 4))) ? 2 : 1;
        for (int I = J + (wv - fw0); I < 8; I += 4 - fw0) {
          const int tb = bidx(I, J - 1) * 256;
#pragma unroll
          for (int q = 0; q < 4; ++q) st_sc1(&pubL[tb + q * 64 + lane], sD[tb + q * 64 + lane]);
        }
      }
      // V & 512: wave 2 writes the whole block column back, so that wave 3's store wait (its
      // vmcnt(0) before the barrier) covers only its Dinv stores
      // (V & 262144: no write-back here -- nothing in the launch reads L11 from A; it goes back
      // after the role's last progress word, off the chain)
      if (V & 262144) {
      } else if (V & 512) {
        if (wv == 2) write_back(J - 1, 0, 1);
      } else if (wv >= 2) {
        write_back(J - 1, wv - 2, 2);
      }
      STAMPAT(64 + 8 * wv + J);
      // free waves: {1, 2, 3} or {2, 3}; tile I = J+1.. round robin.  V & 128: wave 3 (the
      // inverse, ~3900 cycles) takes no look-ahead tiles -- they go to the other free waves
      const int f0 = (ONE ? nbt > 3 : (nbt > 4 || (DL && nbt == 4))) ? 2 : 1;
      const int nf = (V & 128) ? 3 - f0 : 4 - f0;
      if (DL) {
        // wave 3 publishes Dinv only (4 stores): all free waves share the tiles round robin
        if (!(V & 8))
          for (int I = J + 1 + (wv - f0); I < 8; I += 4 - f0) tile_update_n(I, J + 1, J);
      } else if (V & 256) {
        // greedy list schedule of the look-ahead tiles I = J+1..7 over the free waves, by cost
        // estimates in cycles (lab stamps): the inverse ~4000 (wave 3), publish + write-back
        // ~1000 (wave 2; publish alone ~300 with the write-back deferred), a tile ~400 + 250 J;
        // every wave computes the same schedule
        int It[6] = {0, 0, 0, 0, 0, 0};
        int nt = 0;
        int load[4] = {1 << 30, f0 <= 1 ? 0 : (1 << 30), (V & 262144) ? 300 : 1000, 4000};
        for (int I = J + 1; I < 8; ++I) {
          int best = 1;
#pragma unroll
          for (int w = 2; w < 4; ++w)
            if (load[w] < load[best]) best = w;
          load[best] += 400 + 250 * J;
          if (best == wv) It[nt++] = I;   // at most 7 - J <= 6 tiles
        }
        if (!(V & 8))
          for (int t0 = 0; t0 < nt; t0 += 3)
            tile_update_multi(It + t0, (1u << std::min(3, nt - t0)) - 1u, J + 1, J);
      } else if ((V & 1048576) && f0 == 2) {
        // iterations with two leaf waves (J <= 2): wave 3 (the inverse) also takes the last tile
        if (!(V & 8) && wv >= 2)
          for (int I = (wv == 3 ? 7 : J + 1); I < (wv == 3 ? 8 : 7); ++I) tile_update_n(I, J + 1, J);
      } else if (!(V & 8) && !((V & 128) && wv == 3)) {
        for (int I = J + 1 + (wv - f0); I < 8; I += nf) tile_update_n(I, J + 1, J);
      }
      STAMPAT(80 + 8 * wv + J);
    }
    if (pubL) {
      if ((V & 1) && leafw) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");   // the previous leaf's rows
      else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    __syncthreads();
    STAMP();
    if (fail) break;
    // block row J-1 of L11 and Dinv_{J-1} are stored: release them to the row workgroups
    if (pubL && tid == 0 && J > 0) __hip_atomic_store(progress, (unsigned)J, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    STAMP();
  }
  if (fail) {
    if (tid == 0) {
      atomicCAS(info, 0, (int)(k0 + fail));
      __threadfence();   // (info before the failure word: a waiter released by failw cannot report first)
      if (failw) atomicCAS(failw, 0u, (unsigned)(k0 + fail));
      // release the row workgroups (they finish on garbage; the failed factor is discarded)
      if (pubL) {
        __threadfence();
        __hip_atomic_store(progress, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  {
    const int Jl = nJ - 1;   // the last block column (7 for a full panel)
    if (wv == 3) {
      if (V & 2097152) publish_dinv(&sm.sdinv[(Jl & 1) * 256], dinv_out + Jl * 256, lane, pubL != nullptr);
      else tri_inverse16(&sD[bidx(Jl, Jl) * 256], &srinv[Jl * 16], dinv_out + Jl * 256, lane, pubL != nullptr);
    }
    if (wv == 2 && pubL) {
      const int db = bidx(Jl, Jl) * 256;
#pragma unroll
      for (int q = 0; q < 4; ++q) st_sc1(&pubL[db + q * 64 + lane], sD[db + q * 64 + lane]);
    }
    if (wv == 1 && !(V & 262144)) write_back(Jl, 0, 1);   // (block columns 0 .. Jl-1 went back during the loop)
  }
  if (pubL) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(progress, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  STAMP();
  if (V & 262144) {
    // L11 back to A after the last progress word: its readers are the backward solve and later
    // launches (the row roles and the fold tiles read pubL / the row chunks' outputs)
    for (int Jc = 0; Jc < nJ; ++Jc) write_back(Jc, wv, 4);
  }
}
#undef STAMP


// control words of one Cholesky launch (k_potrf_block; the header of block_ctl_words)
enum {
  CTL_TICKET = 0, CTL_PA_PROG = 1, CTL_PA_NEXT = 2, CTL_PB_PROG = 3, CTL_FAIL = 4,
  CTL_NF = 9,                         // next-diagonal-block fold tiles done
  CTL_PB0 = 16,                       // P(b)'s first row chunk done (the tail role waits for it)
  CTL_HDR = CTL_PB0 + 1
};

// Row role: rows below the diagonal block, L21 = A21 L11^-T, 64 rows per workgroup, 16 rows per
// wave.  Each wave runs the 8-step block forward substitution in MFMA registers,
//   X_J = (B_J - sum_{P<J} X_P L_JP^T) Dinv_J^T,
// starting step J as soon as the diagonal role has released block row J (*progress > J).
// L blocks and Dinv come from the producer's sc1 stores and are read with sc1 loads only.
// FUSED: as for diag_role; *done (if given) is set once this chunk's rows (and its part of the
// next panel's columns) are stored.  next_nb > 0: the first nchd chunks publish their rows (the
// next panel's diagonal block rows) and every chunk applies this panel to its rows of the next
// panel's columns -- except the publishing chunks when fold_pub is false (the fused kernel folds
// the next diagonal block with separate tile workgroups).
// LDS (VEC, IPM_ROW_LDS): the workgroup stages what its four waves share through LDS with 16-byte
// direct loads (global_load_lds, sc1), all of it in flight at once: the off-diagonal L blocks and
// Dinv of every block row the diagonal role has released (one memory latency when the role is
// already done -- the row chunks of a trailing-bound launch start after its tiles -- instead of
// one per block row), then per half of the fold its 128 x 64 operand and the destination values.
// A chunk that starts after its diagonal role paid ~26 dependent memory latencies before
// (profiles/r6rt: 33 us per P(a) chunk in the tail of launch 16 at n = 8192).  Every value is
// formed by the same operations as the register path.  Off by default: measured slower
// (profiles/r6x/ab3: n = 8193 5.59 -> 5.68 ms, 2048 0.600 -> 0.61 ms; the kernel's SGPR spills
// 16 -> 55, and in chain-bound launches every block row adds a barrier round trip).
#ifndef IPM_ROW_LDS
#define IPM_ROW_LDS 0
#endif
template <bool FUSED = false, bool LDS = false>
__device__ __forceinline__ void row_role(int64_t chunk, int64_t n, int64_t k0, int nb, double* __restrict__ A,
                                         int64_t lda, const double* dinv, const double* pubL,
                                         unsigned* progress, int next_nb, unsigned* nextc, double* stage,
                                         int* sflag, unsigned* done = nullptr, bool fold_pub = true,
                                         int* sinfo = nullptr, unsigned* failw = nullptr, bool sc1_rows = false) {
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int64_t row = k0 + nb + chunk * PF_RB + wv * 16 + fr;
  const bool rin = row < n;
  // prefetch this wave's 16 x 128 slab of A21 (transposed D layout): b_J reg r = B[row][J*16 + fk + 4r]
  double b[8][4];
#pragma unroll
  for (int J = 0; J < 8; ++J)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int c = J * 16 + fk + 4 * r;
      b[J][r] = (rin && c < nb) ? (FUSED ? ld_sc1(&A[(k0 + c) * lda + row]) : A[(k0 + c) * lda + row]) : 0.0;
    }
  dbl4 x[8];
#pragma unroll
  for (int J = 0; J < 8; ++J) x[J] = dbl4{0.0, 0.0, 0.0, 0.0};
  if constexpr (LDS) {
    // sL: off-diagonal block (J, P) at sL[(J (J - 1) / 2 + P) 256], Dinv_J at sL[7168 + 256 J]
    // (9216 doubles: the diagonal role's sD)
    double* sL = stage;
    const int nJ = (nb + 15) >> 4;
    int issued = 0;   // block rows [0, issued) are in LDS (workgroup-uniform)
#pragma unroll
    for (int J = 0; J < 8; ++J) {
      if (J >= nJ) break;
      if (issued <= J) {
        if (tid == 0) {
          // (no bound of its own: see the register path below)
          unsigned kn = ld_ctl(progress);
          while (kn <= (unsigned)J) {
            __builtin_amdgcn_s_sleep(2);
            kn = ld_ctl(progress);
          }
          *sflag = (int)min(kn, 8u);   // 0xFFFFFFFF (failed diagonal): everything, on garbage
        }
        __syncthreads();
        const int upto = min(__builtin_amdgcn_readfirstlane(*sflag), nJ);
        // block row r: 2 r wave instructions of L blocks (1 KB each), then 2 of Dinv_r
        int ins = 0;
        for (int r = issued; r < upto; ++r)
          for (int q = 0; q < 2 * r + 2; ++q, ++ins) {
            if ((ins & 3) != wv) continue;
            const bool lq = q < 2 * r;
            const double* src = lq ? pubL + bidx(r, q >> 1) * 256 + (q & 1) * 128 : dinv + r * 256 + (q - 2 * r) * 128;
            double* dst = lq ? sL + ((r * (r - 1)) / 2 + (q >> 1)) * 256 + (q & 1) * 128
                             : sL + 7168 + r * 256 + (q - 2 * r) * 128;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 2 * lane),
                                             (__attribute__((address_space(3))) void*)dst, 16, 0, 16);   // sc1
          }
        issued = upto;
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
      }
      dbl4 acc = dbl4{b[J][0], b[J][1], b[J][2], b[J][3]};
#pragma unroll
      for (int P = 0; P < J; ++P) {
        const double* lb = sL + ((J * (J - 1)) / 2 + P) * 256 + fk * 16 + fr;
        double av[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) av[s4] = -lb[64 * s4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], x[P][s4], acc, 0, 0, 0);
      }
      const double* ib = sL + 7168 + J * 256 + fk * 16 + fr;
      double dvv[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) dvv[s4] = ib[64 * s4];
      dbl4 xj = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) xj = __builtin_amdgcn_mfma_f64_16x16x4f64(dvv[s4], acc[s4], xj, 0, 0, 0);
      x[J] = xj;
    }
  } else {
  unsigned known = 0;
#pragma unroll
  for (int J = 0; J < 8; ++J) {
    if (16 * J >= nb) break;   // a partial panel's diagonal role stops at its last block column
    // (every lane polls.  No bound of its own -- a wall-clock start held across this loop made the
    // kernel spill registers: the diagonal role it waits for is resident (lower ticket), its only
    // waits are the bounded ones at its start, and after them it always publishes: progress
    // reaches every block row, or 0xFFFFFFFF when the block fails)
    while (known <= (unsigned)J) {
      known = ld_ctl(progress);
      if (known <= (unsigned)J) __builtin_amdgcn_s_sleep(2);
    }
    dbl4 acc = dbl4{b[J][0], b[J][1], b[J][2], b[J][3]};
#pragma unroll
    for (int P = 0; P < J; ++P) {
      const double* lb = pubL + bidx(J, P) * 256 + fk * 16 + fr;
      double av[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) av[s4] = -ld_sc1(lb + 64 * s4);
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], x[P][s4], acc, 0, 0, 0);
    }
    const double* ib = dinv + J * 256 + fk * 16 + fr;
    double dvv[4];
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) dvv[s4] = ld_sc1(ib + 64 * s4);
    dbl4 xj = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) xj = __builtin_amdgcn_mfma_f64_16x16x4f64(dvv[s4], acc[s4], xj, 0, 0, 0);
    x[J] = xj;
  }
  }   // LDS
  // rows of the next panel's diagonal block are handed to the other workgroups of this launch
  const int nchd = (next_nb + PF_RB - 1) / PF_RB;
  const bool pub = chunk < nchd;
  if (rin) {
#pragma unroll
    for (int J = 0; J < 8; ++J)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = J * 16 + fk + 4 * r;
        if (c < nb) {
          // (FUSED: every row write-through, like the published chunks -- the tail workgroup reads
          // the last rows inside this launch, and a plain store would keep the line shared with
          // the neighbouring chunk's rows (an unaligned leading dimension) in this XCD's L2 with
          // that chunk's rows as they were: r6, 4 of 12 runs of the bordered n = 8193 trajectory)
          if (FUSED || pub || sc1_rows) st_sc1(&A[(k0 + c) * lda + row], x[J][r]);
          else A[(k0 + c) * lda + row] = x[J][r];
        }
      }
  }
  if (next_nb > 0 && pub) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(nextc, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // with fold_pub false a publishing chunk still folds its rows BELOW the next diagonal block
  // (they exist when next_nb is not a multiple of PF_RB and rows follow it, e.g. the bordered
  // right-hand-side row of the Newton factorization)
  const int64_t nd_end = k0 + nb + next_nb;
  const bool fold_chunk = fold_pub || !pub || (k0 + nb + (chunk + 1) * PF_RB > nd_end && nd_end < n);
  const bool rfold = rin && (fold_pub || !pub || row >= nd_end);
  if (next_nb > 0 && fold_chunk) {
  // ---- fused intra-block update (replaces a GEMM launch between the two panels of a block):
  //   A[rows, k0+nb : k0+nb+next_nb] -= X[rows, :] L[k0+nb : k0+nb+next_nb, k0 : k0+nb]^T
  // (nb == 128 here).  The second factor is this panel's result for the first nchd row chunks.
  if (tid == 0) {
    int ok = 1;
    spin_until<2>(sinfo, failw, [&] {
      if (ld_ctl(nextc) >= (unsigned)nchd) return true;
      if (ld_ctl(progress) == 0xFFFFFFFFu) { ok = 0; return true; }   // diagonal failed: info is set
      return false;
    });
    *sflag = ok;
  }
  __syncthreads();
  constexpr int SLAB = 128 * 16 + 16;   // one 16-row slab of the second factor, k-major (+ bank pad)
  if constexpr (LDS) {
    // per half h: the 4 slabs (16 columns each) as 64 wave instructions of 8 k rows x 16 columns,
    // and the 16 destination values of this lane, all in flight before one wait
    const bool go = *sflag != 0;
#pragma unroll 1
    for (int h = 0; h < 2 && go; ++h) {
      if (64 * h >= next_nb) break;
      __syncthreads();   // (h = 0: the TRSM's LDS reads and *sflag are done; h = 1: the last half's)
      for (int i = wv; i < 64; i += 4) {
        const int jl = i >> 4, kk = (i & 15) * 8 + (lane >> 3), jp = 16 * jl + 2 * (lane & 7);
        if (64 * h + jp < next_nb) {
          const double* src = A + (k0 + kk) * lda + k0 + nb + 64 * h + jp;
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                           (__attribute__((address_space(3))) void*)(stage + jl * SLAB + (i & 15) * 128),
                                           16, 0, 16);   // sc1
        }
      }
      double cv[4][4];
#pragma unroll
      for (int jl = 0; jl < 4; ++jl)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int c = 64 * h + 16 * jl + fk + 4 * r;
          cv[jl][r] = (rfold && c < next_nb) ? ld_sc1(&A[(k0 + nb + c) * lda + row]) : 0.0;
        }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
#pragma unroll
      for (int jl = 0; jl < 4; ++jl) {
        const int jt = 4 * h + jl;
        if (16 * jt >= next_nb) break;
        const int64_t col0 = k0 + nb + 16 * jt;
        dbl4 acc = dbl4{cv[jl][0], cv[jl][1], cv[jl][2], cv[jl][3]};
        const double* sb = stage + jl * SLAB + fk * 16 + fr;
#pragma unroll
        for (int P = 0; P < 8; ++P)
#pragma unroll
          for (int s4 = 0; s4 < 4; ++s4)
            acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-sb[(16 * P + 4 * s4) * 16], x[P][s4], acc, 0, 0, 0);
        if (rfold) {
#pragma unroll
          for (int r = 0; r < 4; ++r)
            if (16 * jt + fk + 4 * r < next_nb) st_sc1(&A[(col0 + fk + 4 * r) * lda + row], acc[r]);
        }
      }
    }
  } else {
#pragma unroll 1
  for (int h = 0; h < 2 && *sflag; ++h) {
    if (64 * h >= next_nb) break;
    if (h) __syncthreads();
    {
      // thread (k = wv + 4q, jj = lane): 512 contiguous bytes per wave and k
      const bool jin = 64 * h + lane < next_nb;
      const double* src = A + (k0 + wv) * lda + k0 + nb + 64 * h + lane;
      double* dst = stage + (lane >> 4) * SLAB + wv * 16 + (lane & 15);
#pragma unroll 1
      for (int q0 = 0; q0 < 32; q0 += 8) {
        double v[8];
#pragma unroll
        for (int q = 0; q < 8; ++q) v[q] = jin ? ld_sc1(src + (int64_t)(4 * (q0 + q)) * lda) : 0.0;
#pragma unroll
        for (int q = 0; q < 8; ++q) dst[(q0 + q) * 64] = v[q];
      }
    }
    __syncthreads();
#pragma unroll 1
    for (int jl = 0; jl < 4; ++jl) {
      const int jt = 4 * h + jl;
      if (16 * jt >= next_nb) break;
      const int64_t col0 = k0 + nb + 16 * jt;
      dbl4 acc;
#pragma unroll
      for (int r = 0; r < 4; ++r)
        acc[r] = (rfold && 16 * jt + fk + 4 * r < next_nb)
                     ? (FUSED ? ld_sc1(&A[(col0 + fk + 4 * r) * lda + row]) : A[(col0 + fk + 4 * r) * lda + row])
                     : 0.0;
      const double* sb = stage + jl * SLAB + fk * 16 + fr;
#pragma unroll
      for (int P = 0; P < 8; ++P)
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4)
          acc = __builtin_amdgcn_mfma_f64_16x16x4f64(-sb[(16 * P + 4 * s4) * 16], x[P][s4], acc, 0, 0, 0);
      if (rfold) {
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (16 * jt + fk + 4 * r < next_nb) {
            if (FUSED) st_sc1(&A[(col0 + fk + 4 * r) * lda + row], acc[r]);
            else A[(col0 + fk + 4 * r) * lda + row] = acc[r];
          }
      }
    }
  }
  }   // LDS
  }   // next_nb > 0
  if (done) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(done, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
}

// =====================================================================================
// One launch per 256-column block (default path).  Block b = columns [cb, cb + wa + wbw):
//   LA  tiles : A[cb:n, block b] -= L[cb:n, block b-1] L[block b, block b-1]^T   (64-tiles,
//               row blocks in order; la_done[row block] counts finished tiles)
//   P(a)      : panel [cb, cb+wa): diagonal role, then row chunks; the row chunks also apply
//               P(a) to P(b)'s columns (fold) and set pa_done[chunk]
//   P(b)      : panel [cb+wa, cb+wa+wbw) (waits for pa_done of the chunks holding its rows)
//   S   tiles : A[cb+wb:n, cb+wb:n] -= L[.., block b-1] L[.., block b-1]^T  (128-tiles, lower)
// Workgroups take TICKETS in this order and only ever wait for lower tickets, so the launch
// cannot deadlock for any residency (and not beside other launches either).  Everything one
// workgroup hands to another inside the launch moves with sc1 loads/stores.
// The panel work of block b thus overlaps the trailing update of block b-1 in ONE stream: no
// cross-stream event waits (~10 us each on this platform).
// =====================================================================================
struct BlockArgs {
  int64_t n = 0, lda = 0;
  double* A = nullptr;
  int* info = nullptr;
  double* wsA = nullptr;        // P(a): Dinv (PF_DINV) + packed L11 (36 blocks)
  double* wsB = nullptr;        // P(b): same
  unsigned* ctl = nullptr;      // this launch's zeroed control words (CTL_* below)
  const unsigned* prevfail = nullptr;   // failure word of the previous launch
  int64_t cb = 0;
  int wa = 0, wbw = 0;
  int nla = 0, nra = 0, nrb = 0, la_tj = 0, nlab = 0;
  int64_t ns = 0;
  int nnf = 0;                  // next-diagonal-block fold tiles (32 x 32, lower triangle)
  GemmArgs la32, la, la128, s;   // look-ahead: 32-tiles (rows, cols < 128, lower), 64-tiles (rows
                                 // 128..255, or all rows >= 128 below IPM_LA128_MIN), 128-tiles (rows >= 256)
  int nla32 = 0, la32_T = 0, nla64 = 0, nla128 = 0;
  int trace = 0;                // IPM_ROLE_TRACE builds: record this launch's roles
  // ragged trailing rows (IPM_RAG, default on): the last rag_n <= 8 rows of the trailing update,
  // [rag_r0, rag_r0 + rag_n) relative to its origin, are updated by nrag row workgroups (one
  // K = 256 dot product per element) instead of a row of 128-tiles (the bordered Newton system
  // has 1-2 rows past a multiple of 128)
  int64_t rag_r0 = 0;
  int rag_n = 0, nrag = 0;
  // trailing tiles split in two K halves (the planner's pick for the launch's last round):
  // S tickets [0, s_full) are whole tiles, then two per split tile (tile s_full + p)
  int64_t s_full = 0;
  double* sscr = nullptr;       // split p's upper-half partial tile at sscr + p * 128 * 128
  unsigned* sflag = nullptr;    // split p done: sflag[p]
  // block pairs (IPM_PAIR, potrf_pair_plan): the trailing tiles apply TWO earlier blocks at once
  // (K = 512: C read and written once per 512 columns of L instead of per 256).  S tickets
  // [0, nstrip) are the strip tiles (s2: the next block's 256 columns, 2 tiles per tile row); the
  // rest index the far-region tile list of s from f0 on (a pair's two launches each take a part).
  int64_t nstrip = 0, f0 = 0;
  GemmArgs s2;
  int rag_K = CH_NB;            // ragged rows: K extent and first column of the applied blocks
  int64_t rag_cp = 0;
  // tail (potrf_plan): the factorization's last tail_r <= 8 columns (tail_R <= 16 rows from tail_o
  // on, the bordered right-hand-side row included) are finished by ONE workgroup of the launch
  // before them instead of a launch of their own: it applies L's columns [tail_k0, tail_k0 +
  // tail_K) to the corner and factors it
  int ntail = 0, tail_r = 0, tail_R = 0, tail_K = 0;
  int64_t tail_o = 0, tail_k0 = 0;
};
// this workgroup's compute unit: XCC id, SE / SH / CU ids from HW_ID
__device__ __forceinline__ unsigned cu_key() {
  const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
  const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
  return ((xcc & 15u) << 8) | ((hw >> 8) & 0xFFu);
}
// control words per launch (block_ctl_words, ipm_common.h): header, la_done[ceil(n/64)],
// pa_done[ceil(n/64)]

union BlockSmem {
  DiagSmem d;
  MfSmem<128, 2> g128;
  MfSmem<64, 2> g64;
  MfSmem<32, 2> g32;
};

// thread 0 waits until words w[0..cnt) are all >= target (or the bound runs out); then the
// workgroup proceeds
__device__ __forceinline__ void wait_words(unsigned* w, int cnt, unsigned target, int* info, unsigned* failw) {
  if (threadIdx.x == 0)
    for (int i = 0; i < cnt; ++i)
      if (!spin_until<2>(info, failw, [&] { return ld_ctl(w + i) >= target; })) break;
  __syncthreads();
}

#ifdef IPM_ROLE_TRACE
// diagnostic build only: per workgroup of the traced launch {ticket | role << 32, start, end}
// in s_memrealtime ticks (100 MHz)
__device__ unsigned long long ipm_role_trace[8192 * 4];
struct RoleTrace {
  bool on;
  int ticket;
  unsigned long long t0;
  int role = -1;
  // (NF fold tiles: wake = the spin's end, loaded = operands in registers; recorded instead of the
  // ticket / CU key words)
  unsigned long long wake = 0, loaded = 0;
  __device__ RoleTrace(bool o, int t) : on(o && t < 8192), ticket(t), t0(__builtin_amdgcn_s_memrealtime()) {}
  __device__ ~RoleTrace() {
    if (on && threadIdx.x == 0) {
      const unsigned lo = wake ? (unsigned)(loaded - t0) : (unsigned)ticket;
      ipm_role_trace[4 * ticket] = (unsigned long long)lo | ((unsigned long long)(unsigned)role << 32);
      ipm_role_trace[4 * ticket + 1] = t0;
      ipm_role_trace[4 * ticket + 2] = __builtin_amdgcn_s_memrealtime();
      ipm_role_trace[4 * ticket + 3] = wake ? wake : cu_key();
    }
  }
};
#define ROLE(r) (rt.role = (r))
#define ROLE_STAMP(f) (rt.f = __builtin_amdgcn_s_memrealtime())
// fold tiles of the traced launch (slots 0-15 look-ahead, 16-31 NF): [slot][0] start, 1 wake,
// 2 + 2p operands of pass p in LDS, 3 + 2p its MFMAs done, 10 stores done, 11 fnp  (s_memrealtime)
__device__ unsigned long long ipm_fold_trace[32 * 12];
#define FOLD_SLOT ((frole == 0 ? 0 : 16) + ftile)
#define FOLD_STAMP(i) do { if (rt.on && ftile < 16 && tid == 0) ipm_fold_trace[FOLD_SLOT * 12 + (i)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define FOLD_STAMP(i) do {} while (0)
#define ROLE(r) ((void)0)
#define ROLE_STAMP(f) ((void)0)
#endif

// FASTS: every trailing tile of this launch is a full 128-tile (K = 256): they run the
// branch-free slab loop (mfma_tile LOOP 1) -- one instantiation per kernel, as the allocator needs
// LAZY (default; IPM_LAZYC=0 turns it off.  FASTS launches whose trailing tiles are all whole K = 256 tiles, no strips or
// K halves): the tiles read C one MFMA block per slab (mfma_tile LAZYC) instead of a 128 KB burst
// before the first MFMA
// The roles of one launch for the workgroup holding launch-local ticket t (see the ticket order
// below).
template <bool VEC, bool FASTS, int LAZY>
__device__ __forceinline__ void potrf_block_body(const BlockArgs& b, int64_t t, BlockSmem& sm, int& sflag) {
  const int tid = threadIdx.x;
  unsigned* const failw = &b.ctl[CTL_FAIL];
#ifdef IPM_ROLE_TRACE
  RoleTrace rt(b.trace != 0, (int)t);
#endif
  // a failure in an earlier launch: pass it on and stop (consistent for every workgroup: the
  // word was final before this launch started).  The look-ahead fold tiles test it after their
  // first operand loads are in flight (the word's latency hidden behind theirs).
  // (r5q trace: the test's load, waited for at once to branch on, held every workgroup ~1.2 us at
  // the launch start)
  const int64_t t_launch = t;
  auto prev_failed = [&]() {
    const unsigned pf = ld_ctl(const_cast<unsigned*>(b.prevfail));
    if (pf == 0) return false;
    if (t_launch == 0 && tid == 0) __hip_atomic_store(&b.ctl[CTL_FAIL], pf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return true;
  };
  if (!(VEC && t < b.nla32 && (b.la32.K % 128) == 0) && prev_failed()) return;
  unsigned* la_done = b.ctl + CTL_HDR;
  unsigned* pa_done = la_done + (b.n + 63) / 64;
  // look-ahead tiles: the first 128 rows x 128 columns (what the P(a) diagonal role waits for,
  // lower part only) as 32 x 32 tiles -- ten short tiles instead of three 64-tiles on the chain --
  // then 64-tiles for rows >= 128.  la_done[64-row block] counts finished tiles of that block.
  // fold tiles (K_NF below): the look-ahead 32-tiles of the P(a) diagonal block -- what its
  // diagonal role waits for, on the chain -- and the tiles folding P(a) into P(b)'s diagonal block
  // run ONE code path: every operand of a K = 128 pass staged in LDS by 16-byte direct loads, then
  // a register MFMA chain (a second inlined copy of it cost the r4w kernel its register allocation)
  int64_t fo = 0, fsrc = 0;            // destination block origin (rows = columns), first source column
  int fni = 0, fnj = 0, fnp = 0;       // destination rows / columns (<= 128), K passes of 128 columns
  int ftile = 0, frole = 9;            // tile in the lower-triangle enumeration, trace role
  unsigned* fdone = nullptr;           // completion counter
  bool fwait = false;                  // wait for P(a)'s published rows of P(b)'s diagonal block
  const bool la_fold = VEC && t < b.nla32 && (b.la32.K % 128) == 0;
  if (t < b.nla && !la_fold) {
    ROLE(0);
    int64_t rb;
    if (t < b.nla32) {
      mfma_tile<32, false, VEC, 2, true>(b.la32, t, sm.g32);
      int64_t i = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);   // tri row of tile t
      while ((i + 1) * (i + 2) / 2 <= t) ++i;
      while (i * (i + 1) / 2 > t) --i;
      rb = i >> 1;
    } else if (t - b.nla32 < b.nla64) {
      const int64_t t64 = t - b.nla32;
      mfma_tile<64, false, VEC, 2, true>(b.la, t64, sm.g64);
      rb = 2 + t64 / b.la_tj;
    } else {
      // rows >= 256: 128-tiles (only the later P(a) row chunks wait for them); two 64-row blocks
      const int64_t t128 = t - b.nla32 - b.nla64;
      mfma_tile<128, false, VEC, 2, true>(b.la128, t128, sm.g128);
      rb = 4 + 2 * (t128 / b.la128.tiles_j);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0 && rb + 1 < b.nlab)
        __hip_atomic_fetch_add(&la_done[rb + 1], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_fetch_add(&la_done[rb], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (la_fold) {
    int64_t i = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);   // tri row of tile t
    while ((i + 1) * (i + 2) / 2 <= t) ++i;
    while (i * (i + 1) / 2 > t) --i;
    fo = b.cb;
    fni = (int)b.la32.ni;
    fnj = (int)b.la32.nj;
    fsrc = b.cb - b.la32.K;
    fnp = (int)(b.la32.K / 128);
    ftile = (int)t;
    frole = 0;
    fdone = &la_done[i >> 1];
  }
  t -= b.nla;
  // LA row blocks [r0/64, r1/64] (rows relative to cb) finished
  auto wait_la = [&](int64_t r0, int64_t r1) {
    if (b.nla == 0) return;
    const int64_t q0 = r0 / 64, q1 = std::min<int64_t>(r1 / 64, b.nlab - 1);
    if (threadIdx.x == 0)
      for (int64_t q = q0; q <= q1; ++q) {
        // tiles per 64-row block: 32-tile tri rows 2q, 2q+1 (q < 2), one row of 64-tiles (q < 4
        // or without 128-tiles), else one row of 128-tiles
        unsigned tgt = (q < 4 || b.nla128 == 0) ? (unsigned)b.la_tj : (unsigned)b.la128.tiles_j;
        if (q < 2) {
          tgt = 0;
          for (int64_t i = 2 * q; i < 2 * q + 2 && i < b.la32_T; ++i) tgt += (unsigned)(i + 1);
        }
        if (!spin_until<2>(b.info, failw, [&] { return ld_ctl(la_done + q) >= tgt; })) break;
      }
    __syncthreads();
  };
  const int64_t k1 = b.cb + b.wa;
  // ticket order after the LA tiles: P(a) diagonal, the P(a) row chunks holding P(b)'s diagonal
  // block rows (nchd), the tiles folding P(a) into that block (NF), P(b) diagonal, ragged-row
  // workgroups, S tiles, the other P(a) row chunks, P(b) row chunks.  Row chunks spin while their
  // diagonal role works; dispatched after the S tiles they do not hold slots the trailing update
  // could use.  Decode first, then ONE call site per role (each role's code is inlined once:
  // register pressure and code size).
  const int nchd = b.wbw > 0 ? (b.wbw + PF_RB - 1) / PF_RB : 0;
  enum { K_DIAG, K_ROW, K_NF, K_TILE, K_RAG, K_TAIL, K_NONE } kind = K_NONE;
  bool pb = false;       // the role belongs to P(b)
  int64_t chunk = 0;
  if (la_fold) {
    kind = K_NF;
  } else if (t == 0) {
    kind = K_DIAG;
  } else if ((t -= 1) < nchd) {
    kind = K_ROW;
    chunk = t;
  } else if ((t -= nchd) < b.nnf) {
    kind = K_NF;
    fo = k1;
    fni = fnj = b.wbw;
    fsrc = b.cb;
    fnp = 1;
    ftile = (int)t;
    fdone = &b.ctl[CTL_NF];
    fwait = true;
  } else {
    t -= b.nnf;
    if (b.wbw > 0 && t == 0) {
      kind = K_DIAG;
      pb = true;
    } else {
      if (b.wbw > 0) t -= 1;
      const int64_t na = b.nra - nchd;
      if (t < b.nrag) {
        kind = K_RAG;
      } else if ((t -= b.nrag) < b.ns) {
        kind = K_TILE;
      } else if ((t -= b.ns) < na) {
        kind = K_ROW;
        chunk = nchd + t;
      } else if ((t -= na) < b.nrb) {
        kind = K_ROW;
        pb = true;
        chunk = t;
      } else if ((t -= b.nrb) < b.ntail) {
        kind = K_TAIL;
      }
    }
  }
  double* ws = pb ? b.wsB : b.wsA;
  unsigned* prog = &b.ctl[pb ? CTL_PB_PROG : CTL_PA_PROG];
  const int64_t kp = pb ? k1 : b.cb;
  const int nbp = pb ? b.wbw : b.wa;
  if (kind == K_DIAG) {
    ROLE(pb ? 3 : 1);
    if (pb) wait_words(&b.ctl[CTL_NF], 1, (unsigned)b.nnf, b.info, failw);
    else wait_la(0, b.wa - 1);
    // (the round-4 one-sweep role, tools/diag2_lab.hip + ipm_diag2.h, ran 5 % faster alone but not
    // inside the launch, and instantiating it here raised the kernel's SGPR spills 80 -> 700+)
#ifdef IPM_ROLE_TRACE
    diag_role<true, IPM_DIAG_V>(kp, nbp, b.A, b.lda, ws, b.info, ws + PF_DINV, prog, sm.d, &b.ctl[CTL_FAIL],
                                b.trace != 0 && !pb);
#else
    diag_role<true, IPM_DIAG_V>(kp, nbp, b.A, b.lda, ws, b.info, ws + PF_DINV, prog, sm.d, &b.ctl[CTL_FAIL], false);
#endif
    return;
  }
  if (kind == K_ROW) {
    ROLE(pb ? 6 : (chunk < nchd ? 2 : 5));
    if (pb) {
      // rows relative to k1 = P(a)'s row origin: the P(a) chunks holding them are done
      const int64_t r0 = b.wbw + chunk * PF_RB;
      const int64_t q1 = std::min<int64_t>((std::min<int64_t>(r0 + PF_RB, b.n - k1) - 1) / PF_RB, b.nra - 1);
      wait_words(pa_done + r0 / PF_RB, (int)(q1 - r0 / PF_RB + 1), 1u, b.info, failw);
    } else {
      const int64_t r0 = b.wa + chunk * PF_RB;
      wait_la(r0, std::min<int64_t>(r0 + PF_RB, b.n - b.cb) - 1);
    }
    row_role<true, VEC && IPM_ROW_LDS>(chunk, b.n, kp, nbp, b.A, b.lda, ws, ws + PF_DINV, prog, pb ? 0 : b.wbw, &b.ctl[CTL_PA_NEXT],
                   sm.d.sD, &sflag, pb ? (chunk == 0 && b.ntail ? &b.ctl[CTL_PB0] : nullptr) : &pa_done[chunk], false,
                   b.info, failw, b.ntail && (b.tail_o - (kp + nbp)) / PF_RB == chunk);
    return;
  }
  if (kind == K_NF) {
    ROLE(frole);
    // destination block D (rows / columns fo.., fni x fnj, lower) -= L L^T over the fnp source
    // column passes [fsrc + 128 p, fsrc + 128 p + 128): one 32 x 32 lower tile per workgroup,
    // 16 x 16 per wave.  NF: D = P(b)'s diagonal block, L = P(a)'s rows of it (published by the
    // first nchd row chunks, fwait).  Look-ahead: D = P(a)'s diagonal block, L = the previous
    // block's (or pair's) columns of its rows, final since the previous launch.
    int ti = 0, q = ftile;
    while (q > ti) { q -= ti + 1; ++ti; }   // ftile -> (ti, tj = q), tj <= ti
    const int tj = q;
    if (fwait) {
      if (tid == 0)
        spin_until<2>(b.info, failw, [&] {
          return ld_ctl(&b.ctl[CTL_PA_NEXT]) >= (unsigned)nchd || ld_ctl(&b.ctl[CTL_PA_PROG]) == 0xFFFFFFFFu;
        });
      __syncthreads();
    }
    ROLE_STAMP(wake);
#ifdef IPM_ROLE_TRACE
    if (rt.on && ftile < 16 && tid == 0) {
      ipm_fold_trace[FOLD_SLOT * 12] = rt.t0;
      ipm_fold_trace[FOLD_SLOT * 12 + 11] = (unsigned long long)fnp;
    }
#endif
    FOLD_STAMP(1);
    const int lane = tid & 63, wv = tid >> 6, fr = lane & 15, fk = lane >> 4;
    const int ib = 32 * ti + 16 * (wv & 1), jb = 32 * tj + 16 * (wv >> 1);
    const bool live = ib + 15 >= jb;   // sub-tiles entirely above the diagonal are never read
    const int i = ib + fr;
    const bool iin = i < fni, jin = jb + fr < fnj;
    double* const D = b.A + fo * b.lda + fo;   // D(i, j) at D[j * lda + i]
    dbl4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int j = jb + fk + 4 * r;
      acc[r] = (live && iin && j < fnj) ? ld_sc1(&D[j * b.lda + i]) : 0.0;
    }
    if constexpr (VEC) {
      // per pass, the two 32-row blocks of L (rows 32 tj.. for the A operand, 32 ti.. for B; the
      // pass's 128 columns) go to LDS with 16-byte direct loads: one wave instruction = 4 columns x
      // 32 rows (lane l: rows 2 (l & 15), +1 of column l >> 4), element (c, r) of block s at
      // sL[4096 s + 32 c + r].  16 instructions per wave instead of 64 8-byte strided loads, which
      // ran past the 63 outstanding loads a wave may hold (r4u trace: 10.7 us from the wake to the
      // operands).  Rows past fni read the next rows / column of the matrix (in bounds) and are
      // masked.
      double* sL = sm.d.sD;
      const int nsrc = ti == tj ? 1 : 2;
      auto issue = [&](int p) {
        for (int it = wv; it < 32 * nsrc; it += 4) {
          const int sblk = it >> 5, c4 = it & 31;
          const int col = 128 * p + 4 * c4 + (lane >> 4);
          const double* src = b.A + (fsrc + col) * b.lda + fo + 32 * (sblk ? ti : tj) + 2 * (lane & 15);
          __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                           (__attribute__((address_space(3))) void*)&sL[sblk * 4096 + c4 * 128], 16,
                                           0, 16);   // aux 16 = sc1
        }
      };
      const double* sa = sL + 16 * (wv >> 1) + fr;                          // L[jb + fr][k] at sa[32 k]
      const double* sbp = sL + (ti == tj ? 0 : 4096) + 16 * (wv & 1) + fr;   // L[i][k]
      // IPM_FOLD_ACC > 1: the MFMA chain over that many accumulators (k interleaved; not bitwise
      // the single-chain sum)
      dbl4 xacc[3] = {dbl4{0.0, 0.0, 0.0, 0.0}, dbl4{0.0, 0.0, 0.0, 0.0}, dbl4{0.0, 0.0, 0.0, 0.0}};
      issue(0);
      if (la_fold && prev_failed()) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // (no LDS writes in flight at exit)
        return;
      }
      // per pass: operands LDS -> registers, then (all waves past a barrier) the next pass's loads
      // go out while this pass's MFMA chain runs from registers.  (r5n trace: with the LDS reads
      // inside the chain a pass's 32 MFMAs took ~3 us, and loads and MFMAs alternated.)
      for (int p = 0; p < fnp; ++p) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        ROLE_STAMP(loaded);
        if (p < 4) FOLD_STAMP(2 + 2 * p);
        // unconditional LDS reads (in bounds; masked rows hold matrix data) and selects after them:
        // a masked read is a branch, and each one waited for its value (64 serialized LDS
        // latencies per pass, ~2 us)
        double av[32], bv[32];
        if (live) {
#pragma unroll
          for (int qq = 0; qq < 32; ++qq) {
            const int k = 4 * qq + fk;
            av[qq] = sa[32 * k];
            bv[qq] = sbp[32 * k];
          }
#pragma unroll
          for (int qq = 0; qq < 32; ++qq) {
            av[qq] = jin ? -av[qq] : 0.0;
            bv[qq] = iin ? bv[qq] : 0.0;
          }
        }
        if (p + 1 < fnp) {
          asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
          __syncthreads();   // every wave holds this pass's operands: the buffer is free
          issue(p + 1);
        }
        if (live) {
#pragma unroll
          for (int qq = 0; qq < 32; ++qq) {
            dbl4& a = (IPM_FOLD_ACC == 1 || qq % IPM_FOLD_ACC == 0) ? acc : xacc[qq % IPM_FOLD_ACC - 1];
            a = __builtin_amdgcn_mfma_f64_16x16x4f64(av[qq], bv[qq], a, 0, 0, 0);
          }
        }
#ifdef IPM_ROLE_TRACE
        if (p < 4) { asm volatile("s_nop 0" ::"v"(acc[0])); FOLD_STAMP(3 + 2 * p); }
#endif
      }
      if (IPM_FOLD_ACC == 2) acc = acc + xacc[0];
      if (IPM_FOLD_ACC == 4) acc = (acc + xacc[0]) + (xacc[1] + xacc[2]);
    } else if (live) {
      // (NF only: unaligned operands never take the look-ahead path above)
      const double* pa = b.A + fsrc * b.lda + fo + jb + fr;   // L[jb + fr][k] at pa[k * lda]
      const double* pbp = b.A + fsrc * b.lda + fo + i;        // L[i][k]
      // all 64 operand loads in flight at once (one latency, not eight)
      double av[32], bv[32];
#pragma unroll
      for (int qq = 0; qq < 32; ++qq) {
        const int64_t k = 4 * qq + fk;
        av[qq] = jin ? -ld_sc1(pa + k * b.lda) : 0.0;
        bv[qq] = iin ? ld_sc1(pbp + k * b.lda) : 0.0;
      }
#pragma unroll
      for (int qq = 0; qq < 32; ++qq) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[qq], bv[qq], acc, 0, 0, 0);
    }
    if (live && iin) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = jb + fk + 4 * r;
        if (j < fnj) st_sc1(&D[j * b.lda + i], acc[r]);
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    FOLD_STAMP(10);
    if (tid == 0) __hip_atomic_fetch_add(fdone, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return;
  }
  if (kind == K_TAIL) {
    ROLE(13);
    // the corner rows [o, o + R) x columns [o, o + r): C -= L L^T over columns [k0, k0 + K) (the
    // previous block's, final since the previous launch, and this launch's, final once P(b)'s
    // first row chunk -- the last rows' -- is done), then a left-looking Cholesky of its r columns
    // with the diagonal role's pivot factor (L_jj = piv dv, L_ij = v dv, dv = rsqrt_pivot(piv))
    wait_words(&b.ctl[CTL_PB0], 1, 1u, b.info, failw);
    const int R = b.tail_R, r = b.tail_r, K = b.tail_K;
    const int64_t o = b.tail_o, k0 = b.tail_k0, lda = b.lda;
    double* Ls = sm.d.sD;        // Ls[i K + k] = L(o + i, k0 + k)
    double* Cs = Ls + R * K;     // Cs[i r + j]: the updated corner, then L
    double* Ts = Cs + R * r;     // one column's values
    for (int e = tid; e < R * K; e += 256) {
      const int k = e / R, i = e - k * R;
      Ls[i * K + k] = ld_sc1(&b.A[(k0 + k) * lda + o + i]);
    }
    __syncthreads();
    for (int p0 = 0; p0 < R * r; p0 += 16) {   // 16 lanes per (i, j), fixed-order reduction
      const int p = p0 + (tid >> 4), q = tid & 15, i = p / r, j = p - i * r;
      const bool live = p < R * r && j <= i;
      double acc = 0.0;
      if (live)
        for (int k = q; k < K; k += 16) acc = fma(Ls[i * K + k], Ls[j * K + k], acc);
#pragma unroll
      for (int m = 8; m >= 1; m >>= 1) acc += __shfl_xor(acc, m, 16);
      if (live && q == 0) Cs[i * r + j] = ld_sc1(&b.A[(o + j) * lda + o + i]) - acc;
    }
    __syncthreads();
    int fcol = 0;
    for (int j = 0; j < r; ++j) {
      if (tid >= j && tid < R) {
        double v = Cs[tid * r + j];
        for (int k = 0; k < j; ++k) v = fma(-Cs[tid * r + k], Cs[j * r + k], v);
        Ts[tid] = v;
      }
      __syncthreads();
      const double piv = Ts[j], dv = rsqrt_pivot(piv);
      if (!(piv > 0.0) && fcol == 0) fcol = j + 1;
      if (tid >= j && tid < R) Cs[tid * r + j] = tid == j ? piv * dv : Ts[tid] * dv;
      __syncthreads();
    }
    if (tid < R)
      for (int j = 0; j < r && j <= tid; ++j) b.A[(o + j) * lda + o + tid] = Cs[tid * r + j];
    if (fcol && tid == 0) {
      atomicCAS(b.info, 0, (int)(o + fcol));
      __hip_atomic_store(failw, (unsigned)(o + fcol), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return;
  }
  if (kind == K_RAG) {
    ROLE(12);
    // ragged rows i in [r0, r0 + rn) of the trailing update (origin o, K = the previous block's
    // 256 columns): C(i, j) -= sum_k L(i, k) L(j, k) for j <= i; workgroup t takes columns
    // j = 256 t + tid.  Nothing else in this launch touches these elements.
    const int64_t o = b.cb + b.wa + b.wbw, cp = b.rag_cp;
    const int64_t m = b.n - o, r0 = b.rag_r0;
    const int rn = b.rag_n, KR = b.rag_K;   // KR <= 512: rn * KR <= 4096 doubles of sD
    double* xr = sm.d.sD;   // xr[q * KR + k] = L(o + r0 + q, cp + k)
    for (int e = tid; e < rn * KR; e += 256) {
      const int q = e / KR, k = e - q * KR;
      xr[e] = b.A[(cp + k) * b.lda + o + r0 + q];
    }
    __syncthreads();
    const int64_t j = t * 256 + tid;
    if (j < m) {
      double* cj = b.A + (o + j) * b.lda + o + r0;   // C(r0 + q, j) = cj[q]
      double acc[8];
#pragma unroll
      for (int q = 0; q < 8; ++q) acc[q] = (q < rn && j <= r0 + q) ? cj[q] : 0.0;
      const double* xp = b.A + cp * b.lda + o + j;   // L(o + j, cp + k) = xp[k * lda]
#pragma unroll 16
      for (int k = 0; k < KR; ++k) {
        const double xj = xp[k * b.lda];
#pragma unroll
        for (int q = 0; q < 8; ++q)
          if (q < rn) acc[q] = fma(-xj, xr[q * KR + k], acc[q]);
      }
#pragma unroll
      for (int q = 0; q < 8; ++q)
        if (q < rn && j <= r0 + q) cj[q] = acc[q];
    }
    return;
  }
  if (kind == K_TILE) {
    ROLE(4);
    // (Until round 5 a tile that landed on the CU of a running critical-path role handed its tile
    // to a spill word and slept, keeping the slot; the r6 A/B put that at +4 % on the n = 8193
    // factorization -- the sleepers and the spilled tiles ran in the launch tails -- and it went.)
    {
        const int64_t st0 = t;
        // S ticket -> strip tile (pair launches), whole tile, or one K-half of a split tile
        // (pieces: upper half, then lower)
        const bool strip = st0 < b.nstrip;
        const int64_t st = strip ? st0 : st0 - b.nstrip, u = strip ? -1 : st - b.s_full;
        const int sp = u < 0 ? 0 : ((u & 1) ? 2 : 1);
        const int64_t p = u < 0 ? 0 : (u >> 1);
        GemmArgs g = b.s;
        if (strip) {
          g.ni = b.s2.ni;
          g.nj = b.s2.nj;
          g.X = b.s2.X;
          g.Y = b.s2.Y;
          g.C = b.s2.C;
          g.rowmajor = 1;
          g.xcd_remap = 0;
          g.tiles_i = b.s2.tiles_i;
          g.tiles_j = b.s2.tiles_j;
          g.nblk = b.s2.nblk;
        }
        // (both loops in one kernel raised the SGPR spills 89 -> 621 and cost 2.5 %: the launch
        // picks the kernel instead, FASTS)
        mfma_tile<128, false, VEC, 2, false, false, (FASTS && VEC) ? 1 : 0, (FASTS && VEC) ? LAZY : 0>(
            g, strip ? st + (st >= 1 ? 1 : 0) /* (tile (0, 1) lies above the diagonal) */
                     : b.f0 + (u < 0 ? st : b.s_full + p),
            sm.g128, sp, b.sscr + p * (128 * 128), b.sflag + p, -1, -1, b.info, failw);
    }
  }
}

template <bool VEC, bool FASTS = false, int LAZY = 0>
__global__ __launch_bounds__(256, 2) void k_potrf_block(BlockArgs b_arg) {
  IPM_KARGS(BlockArgs, b, b_arg);   // (fields loaded where each role uses them: ipm_mfma.h)
  __shared__ BlockSmem sm;
  __shared__ int sticket, sflag;
  if (threadIdx.x == 0) sticket = (int)atomicAdd(&b.ctl[CTL_TICKET], 1u);
  __syncthreads();
  potrf_block_body<VEC, FASTS, LAZY>(b, __builtin_amdgcn_readfirstlane(sticket), sm, sflag);
}

// workspace: [P(a) Dinv + L11][P(b) Dinv + L11][control words]
static constexpr int64_t PANEL_WS = PF_DINV + 36 * 256;

// zero two word ranges in one launch (replaces two hipMemsetAsync calls on the hot path)
__global__ void k_zero2(unsigned* a, int64_t na, unsigned* b, int64_t nb) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < na) a[i] = 0u;
  else if (i - na < nb) b[i - na] = 0u;
}
// k_zero2 plus the bordered right-hand side (k_border_rhs's row N and corner) in the same launch
__global__ void k_zero2_border(unsigned* a, int64_t na, unsigned* b, int64_t nb, BorderJob j) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < na) a[i] = 0u;
  else if (i - na < nb) b[i - na] = 0u;
  else {
    const int64_t c = i - na - nb;
    if (c < j.N) j.H[c * j.ldh + j.N] = j.scale * j.g[c];
    else if (c == j.N) j.H[j.N * j.ldh + j.N] = j.corner;
  }
}
static void zero2(hipStream_t st, void* a, int64_t na, void* b, int64_t nb) {
  const int64_t tot = na + nb;
  if (tot > 0)
    hipLaunchKernelGGL(k_zero2, dim3((unsigned)cdiv(tot, 256)), dim3(256), 0, st, reinterpret_cast<unsigned*>(a), na,
                       reinterpret_cast<unsigned*>(b), nb);
}

// ---- split planner: how many of a launch's trailing tiles to cut into two K halves.  The
// launch is list-scheduled on the host (2 workgroup slots per CU, items in ticket order, durations
// in units of one 128 x 128 x 256 trailing tile, ~100 us; role durations from the IPM_ROLE_TRACE
// timelines in DESIGN.md): whole tiles 1.0, half tiles 0.55, row chunks 0.5, look-ahead tiles 0.8,
// P(a) / P(b) diagonal roles 0.6 / 1.25.  The q with the smallest makespan wins (0 when the launch
// is chain-bound).  Splitting the LAST q tiles turns a last round that would hold a few whole
// tiles into one of half tiles running on twice as many slots.
static int num_cus();
static double split_makespan(int slots, const std::vector<std::pair<int64_t, double>>& items) {
  std::priority_queue<double, std::vector<double>, std::greater<double>> q;
  for (int i = 0; i < slots; ++i) q.push(0.0);
  double mk = 0.0;
  for (const auto& it : items)
    for (int64_t k = 0; k < it.first; ++k) {
      const double t = q.top() + it.second;
      q.pop();
      q.push(t);
      mk = std::max(mk, t);
    }
  return mk;
}
// (pair launches, K = 512: tiles cost tc = 1.6 (tools/tile_lab.hip: 154 vs 96 us), look-ahead
// tiles twice their K = 256 cost, and the nstrip strip tiles come first)
// S tickets [0, ns_all) = nstrip strips, ns - q whole tiles, 2 q halves; the non-critical row
// chunks (nra of P(a), nrb of P(b)) go before S tickets sa and sb
static std::vector<std::pair<int64_t, double>> launch_items(int64_t nla, int64_t nchd, int64_t nnf, bool pb,
                                                            int64_t nrag, int64_t nstrip, int64_t ns, int64_t q,
                                                            double tc, double lac, int64_t nra, int64_t nrb,
                                                            int64_t sa, int64_t sb) {
  std::vector<std::pair<int64_t, double>> it = {{nla, lac}, {1, 0.6}, {nchd, 0.66}, {nnf, 0.8}, {pb ? 1 : 0, 1.25},
                                                {nrag, 0.1 * tc}};
  // S pieces: [begin, end) in S-ticket index with a duration
  const int64_t e1 = nstrip + ns - q, e2 = e1 + 2 * q;
  auto span = [&](int64_t a, int64_t z) {
    const int64_t w1 = std::max<int64_t>(0, std::min(z, e1) - a);
    const int64_t w2 = std::max<int64_t>(0, std::min(z, e2) - std::max(a, e1));
    if (w1 > 0) it.push_back({w1, tc});
    if (w2 > 0) it.push_back({w2, 0.55 * tc});
  };
  sa = std::min(sa, e2);
  sb = std::min(std::max(sb, sa), e2);
  span(0, sa);
  it.push_back({nra, 0.5});
  span(sa, sb);
  it.push_back({nrb, 0.5});
  span(sb, e2);
  return it;
}
static int64_t plan_split(int64_t nla, int64_t nchd, int64_t nnf, bool pb, int64_t nrag, int64_t ns, int64_t nrows,
                          int64_t cap, double tc = 1.0, int64_t nstrip = 0, double lac = 0.8, int64_t nra = -1,
                          int64_t sa = -1, int64_t sb = -1) {
  if (ns < 64) return 0;
  const int slots = 2 * num_cus();
  if (nra < 0) {   // rows last
    nra = nrows;
    sa = sb = nstrip + ns;
  }
  const int64_t nrb = nrows - nra;
  auto mk = [&](int64_t q) {
    int64_t a = sa, z = sb;
    return split_makespan(slots, launch_items(nla, nchd, nnf, pb, nrag, nstrip, ns, q, tc, lac, nra, nrb, a, z));
  };
  const double m0 = mk(0);
  double best = m0;
  int64_t bq = 0;
  for (int64_t q = 8; q <= std::min(ns, cap); q += 8) {
    const double m = mk(q);
    if (m < best - 0.02) { best = m; bq = q; }
  }
  return bq;
}

// ---- block pairs.  Launch kinds: 0 plain (the trailing update of block b-1 over everything right
// of block b); 2 EVEN e (its look-ahead tiles, the next block's strip and the first f1 tiles of the
// far region F -- everything right of block e+1 -- apply the PAIR e-2, e-1 with K = 512); 1 ODD
// e+1 (look-ahead: block e, K = 256; trailing: the rest of F with the pair e-2, e-1).  The launch
// before the first EVEN is an ODD with nothing to apply (its chain runs without trailing work once);
// the last EVEN takes all of F and plain launches follow.  Pairs run while F has at least
// IPM_PAIR_MIN rows (default 6144: the first, most trailing-bound launches); IPM_PAIR=0 turns them off.
struct PairPlan {
  std::vector<int> kind;      // per 256-column block
  std::vector<int64_t> f1;    // EVEN: F tiles it takes (tile list [0, f1)); ODD: the EVEN's f1
};
static PairPlan potrf_pair_plan(int64_t n, int64_t ncols, int64_t nblocks) {
  PairPlan pl;
  pl.kind.assign(nblocks, 0);
  pl.f1.assign(nblocks, 0);
  // Pairs pay only while the far region is large: at n = 8192 with F >= 3072 rows (five pairs) they
  // were slower, 6.49 -> 6.73 ms (the later pairs' K = 512 tiles fill one round and the row chunks
  // queue behind); F >= 6144 (three pairs, launches 1-6) is the best threshold of the r3 sweep,
  // 6.40 -> 6.22 ms (6656: 6.31, 5632: 6.35; profiles/r3_pair_sweep.txt).  IPM_PAIR=0: off.
  static const bool on = [] { const char* e = getenv("IPM_PAIR"); return !(e && e[0] == '0'); }();
  static const int64_t minrows = [] { const char* e = getenv("IPM_PAIR_MIN"); return e ? atoll(e) : 6144LL; }();
  if (!on || ncols < n - 8) return pl;   // (a partial factorisation keeps the plain order)
  // EVEN e needs block e+1 to exist and F = rows beyond block e+1 of at least minrows
  int64_t last = -1;
  for (int64_t e = 2; e + 1 < nblocks; e += 2) {
    if (n - (e + 2) * CH_NB < minrows) break;
    last = e;
  }
  if (last < 0) return pl;
  pl.kind[1] = 1;                                  // ODD with nothing pending
  for (int64_t e = 2; e <= last; e += 2) {
    pl.kind[e] = 2;
    if (e < last) pl.kind[e + 1] = 1;
  }
  return pl;
}

// wall-clock bounds of the device-side waits: microseconds -> ticks of
// s_memrealtime (hipDeviceAttributeWallClockRate, kHz; 100 MHz on MI355X)
static unsigned long long wall_ticks(unsigned us) {
  static long long khz = -1;
  if (khz < 0) {
    int dev = 0, v = 0;
    hipGetDevice(&dev);
    khz = (hipDeviceGetAttribute(&v, hipDeviceAttributeWallClockRate, dev) == hipSuccess && v > 0) ? v : 100000;
  }
  const unsigned long long t = (unsigned long long)us * (unsigned long long)khz / 1000ull;
  return t > 0 ? t : 1;
}
constexpr unsigned SPIN_US_DEFAULT = 1000000;   // 1 s: no legitimate wait comes near it
// (the device global ipm_spin_ticks, initially 1 s at 100 MHz, on EVERY visible device: a process
// may drive several GPUs.  Every kernel that spins -- the Cholesky, the split / stream-K tiles, the
// backward solve -- is launched from this translation unit, so this TU's copy of the header's
// static global is the one they read.)
static void set_spin_ticks(int which, unsigned us) {
  const unsigned long long t = wall_ticks(us ? us : SPIN_US_DEFAULT);
  int cur = 0, cnt = 0;
  hipGetDevice(&cur);
  if (hipGetDeviceCount(&cnt) != hipSuccess || cnt < 1) cnt = 1;
  for (int d = 0; d < cnt; ++d) {
    if (hipSetDevice(d) != hipSuccess) continue;
    hipMemcpyToSymbol(HIP_SYMBOL(ipm_spin_ticks), &t, sizeof(t), which * sizeof(t), hipMemcpyHostToDevice);
  }
  hipSetDevice(cur);
}
void set_potrf_spin_limit_us(unsigned us) { set_spin_ticks(0, us); }

// One planned launch of the factorization: its arguments, grid and kernel instantiation
// (0 <true,true,1> lazy-C, 1 <true,true,2> pair lazy-C, 2 <true,true> fast loop, 3 <true,false>,
// 4 <false,false>).
struct BlockLaunch {
  BlockArgs b;
  int64_t grid = 0;
  int inst = 4;
};
// every launch of one factorization (potrf_lower_fused's plan); the control words are NOT zeroed
static void potrf_plan(int64_t n, double* A, int64_t lda, int* info, double* ws, int64_t ncols,
                       std::vector<BlockLaunch>& out) {
  out.clear();
  const int64_t nblocks = cdiv(ncols, CH_NB), cw = block_ctl_words(n);
  unsigned* ctl0 = reinterpret_cast<unsigned*>(ws + 2 * PANEL_WS);
  const bool vec = ((lda & 1) == 0) && ((((uintptr_t)A) & 15) == 0);
  // IPM_RAG=0 / 1: ragged trailing rows as a row of 128-tiles / by the ragged-row workgroups (read
  // per call: tests compare both).  Unset: the workgroups above 5120 rows only -- r6, one-box A/B
  // (profiles/r6g/potrf_ragged_rows_ab.txt): the bordered sizes n = 2049 / 3073 / 4097 factor
  // 0.673 / 1.105 / 1.69 -> 0.602 / 1.003 / 1.56 ms as tiles, n = 6145 / 8193 3.14 / 5.54-5.65 ->
  // 3.18 / 5.81-5.83 ms
  const char* erag = getenv("IPM_RAG");
  const bool rag_on = erag ? erag[0] != '0' : n > 5120;
  // IPM_SPLIT=0: no K-split trailing tiles (read per call: tests compare both)
  const char* esp = getenv("IPM_SPLIT");
  const bool split_on = !(esp && esp[0] == '0');
  // IPM_LAZYC=0: no lazy-C trailing tiles (read per call: tests compare both)
  const char* elz = getenv("IPM_LAZYC");
  const bool lazy_on = !(elz && elz[0] == '0');
  const bool lazy2_on = lazy_on && !(elz && elz[0] == '1');   // IPM_LAZYC=1: K = 256 tiles only
  PairPlan pl = potrf_pair_plan(n, ncols, nblocks);
  // a last block of at most 8 columns with at most 16 rows below its origin (the bordered phase-1
  // system: 1 column, 2 rows) is finished inside the launch before it by one tail workgroup: its
  // own launch (look-ahead fold, a diagonal role for one column, the launch boundary) cost ~90 us
  // per factorization (r5u: phase-1 POTRF 0.764 vs 0.672 ms at n = 2048).  IPM_TAIL=0: off.
  const char* etl = getenv("IPM_TAIL");
  const bool tail_on = !(etl && etl[0] == '0');
  int64_t nemit = nblocks;
  int tail_r = 0;
  if (tail_on && nblocks >= 2 && pl.kind[nblocks - 2] == 0) {
    const int64_t cbl = (nblocks - 1) * CH_NB;
    if (ncols - cbl <= 8 && n - cbl <= 16) {
      nemit = nblocks - 1;
      tail_r = (int)(ncols - cbl);
    }
  }
  for (int64_t bk = 0; bk < nemit; ++bk) {
    const int kind = pl.kind[bk];
    const int64_t Kla = kind == 2 ? 2 * CH_NB : CH_NB;   // look-ahead depth (EVEN: the pair)
    BlockArgs b;
    b.n = n;
    b.lda = lda;
    b.A = A;
    b.info = info;
    b.wsA = ws;
    b.wsB = ws + PANEL_WS;
    b.ctl = ctl0 + 8 + bk * cw;
    b.prevfail = bk == 0 ? ctl0 : ctl0 + 8 + (bk - 1) * cw + CTL_FAIL;
    const int64_t cb = bk * CH_NB, wb = std::min<int64_t>(CH_NB, ncols - cb);
    b.cb = cb;
    b.wa = (int)std::min<int64_t>(wb, PF_NB);
    b.wbw = (int)(wb - b.wa);
    if (bk > 0) {
      const int64_t cp = cb - Kla;
      const int64_t ni = n - cb;
      // rows [0, 128) x columns [0, min(128, wb)), lower: 32-tiles (tri enumeration)
      GemmArgs& c = b.la32;
      c.ni = std::min<int64_t>(ni, 128);
      c.nj = std::min<int64_t>(c.ni, std::min<int64_t>(wb, 128));
      c.ni = std::max(c.ni, c.nj);
      c.K = Kla;
      c.X = c.Y = A + cp * lda + cb;
      c.ldx = c.ldy = lda;
      c.C = A + cb * lda + cb;
      c.ldc = lda;
      c.sub = 1;
      c.tri = 1;
      c.xcd_remap = 0;
      c.tiles_i = cdiv(c.ni, 32);
      c.nblk = c.tiles_i * (c.tiles_i + 1) / 2;
      b.nla32 = (int)c.nblk;
      b.la32_T = (int)c.tiles_i;
      // rows [128, 256) x all wb columns: 64-tiles, row blocks in order (P(b)'s diagonal rows: on
      // the chain); rows >= 256: 128-tiles (IPM_LA128=0: 64-tiles throughout)
      static const bool la128_on = [] { const char* e = getenv("IPM_LA128"); return !e || e[0] != '0'; }();
      // 128-tiles only while more than la128_min rows remain below cb: with fewer, the 64-tiles'
      // shorter tiles reach the P(a) row chunks sooner (profiles/r4m: n = 2048 0.864 -> 0.814 ms,
      // 4096 1.97 -> 1.87, 8193 6.23 -> 6.16; IPM_LA128_MIN=<rows>, 0 = always 128-tiles)
      static const int64_t la128_min = [] { const char* e = getenv("IPM_LA128_MIN"); return e ? atoll(e) : 3072LL; }();
      const bool use128 = la128_on && ni > la128_min;
      GemmArgs& a = b.la;
      a.ni = std::max<int64_t>((use128 ? std::min<int64_t>(ni, 256) : ni) - 128, 0);
      a.nj = wb;
      a.K = Kla;
      a.X = A + cp * lda + cb + 128;
      a.Y = A + cp * lda + cb;
      a.ldx = a.ldy = lda;
      a.C = A + cb * lda + cb + 128;
      a.ldc = lda;
      a.sub = 1;
      a.rowmajor = 1;
      a.xcd_remap = 0;
      a.tiles_i = cdiv(a.ni, 64);
      a.tiles_j = cdiv(a.nj, 64);
      a.nblk = a.tiles_i * a.tiles_j;
      b.nla64 = (int)a.nblk;
      if (use128 && ni > 256) {
        GemmArgs& e = b.la128;
        e = a;
        e.ni = ni - 256;
        e.X = A + cp * lda + cb + 256;
        e.C = A + cb * lda + cb + 256;
        e.tiles_i = cdiv(e.ni, 128);
        e.tiles_j = cdiv(e.nj, 128);
        e.nblk = e.tiles_i * e.tiles_j;
        b.nla128 = (int)e.nblk;
      }
      b.nla = b.nla32 + b.nla64 + b.nla128;
      b.la_tj = (int)a.tiles_j;
      b.nlab = (int)cdiv(ni, 64);
      const int64_t m = n - cb - wb;
      b.rag_cp = cb - CH_NB;
      b.rag_K = CH_NB;
      if (m > 0 && kind == 1) {
        // ODD: the rest of the previous EVEN's far region F (origin = this launch's trailing origin),
        // with that EVEN's pair (columns [cb - 3 CH_NB, cb - CH_NB)); its ragged rows were done there
        if (bk >= 1 && pl.kind[bk - 1] == 2) {
          const int64_t me = m + CH_NB;
          const int64_t rn = (rag_on && me > 128 && (me & 127) != 0 && (me & 127) <= 8) ? (me & 127) : 0;
          const int64_t mF = m - rn;
          GemmArgs& g = b.s;
          g.ni = g.nj = mF;
          g.K = 2 * CH_NB;
          g.X = g.Y = A + (cb - 3 * CH_NB) * lda + cb + wb;
          g.ldx = g.ldy = lda;
          g.C = A + (cb + wb) * lda + cb + wb;
          g.ldc = lda;
          g.sub = 1;
          g.tri = 1;
          g.xcd_remap = 1;
          g.tiles_i = cdiv(mF, 128);
          g.nblk = g.tiles_i * (g.tiles_i + 1) / 2;
          b.f0 = pl.f1[bk - 1];
          b.s_full = g.nblk - b.f0;
          b.ns = b.s_full;
        }
      } else if (m > 0 && kind == 2) {
        // EVEN: strip (block bk+1's columns) + the first f1 tiles of F, both with the pair
        // (columns [cb - 2 CH_NB, cb)); ragged rows across the whole trailing width
        int64_t ms = m;
        if (rag_on && m > 128 && (m & 127) != 0 && (m & 127) <= 8) {
          ms = m - (m & 127);
          b.rag_r0 = ms;
          b.rag_n = (int)(m & 127);
          b.nrag = (int)cdiv(m, 256);
          b.rag_cp = cp;
          b.rag_K = (int)Kla;
        }
        const int64_t o = cb + wb, mF = ms - CH_NB;
        GemmArgs& s2 = b.s2;
        s2.ni = ms;
        s2.nj = CH_NB;
        s2.K = Kla;
        s2.X = s2.Y = A + cp * lda + o;
        s2.ldx = s2.ldy = lda;
        s2.C = A + o * lda + o;
        s2.ldc = lda;
        s2.sub = 1;
        s2.tri = 1;
        s2.rowmajor = 1;
        s2.xcd_remap = 0;
        s2.tiles_i = cdiv(ms, 128);
        s2.tiles_j = 2;
        s2.nblk = s2.tiles_i * 2;
        b.nstrip = s2.nblk - 1;   // (tile (0, 1) lies above the diagonal: skipped)
        GemmArgs& g = b.s;
        g = s2;
        g.rowmajor = 0;
        g.ni = g.nj = mF;
        g.X = g.Y = A + cp * lda + o + CH_NB;
        g.C = A + (o + CH_NB) * lda + o + CH_NB;
        g.xcd_remap = 1;
        g.tiles_i = cdiv(mF, 128);
        g.tiles_j = 0;
        g.nblk = g.tiles_i * (g.tiles_i + 1) / 2;
        const bool last = bk + 1 >= nblocks || pl.kind[bk + 1] != 1;
        const int64_t f1 = last ? g.nblk : std::max<int64_t>(0, std::min<int64_t>(g.nblk, (g.nblk - b.nstrip) / 2));
        pl.f1[bk] = f1;
        b.f0 = 0;
        b.s_full = f1;
        b.ns = b.nstrip + f1;
      } else if (m > 0) {
        GemmArgs& g = b.s;
        int64_t ms = m;   // tile rows of the trailing update (ragged rows split off below)
        if (rag_on && m > 128 && (m & 127) != 0 && (m & 127) <= 8) {
          ms = m - (m & 127);
          b.rag_r0 = ms;
          b.rag_n = (int)(m & 127);
          b.nrag = (int)cdiv(m, 256);
        }
        g.ni = g.nj = ms;
        g.K = CH_NB;
        g.X = g.Y = A + cp * lda + cb + wb;
        g.ldx = g.ldy = lda;
        g.C = A + (cb + wb) * lda + cb + wb;
        g.ldc = lda;
        g.sub = 1;
        g.tri = 1;
        g.xcd_remap = 1;   // XCD-contiguous tile runs
        g.tiles_i = cdiv(ms, 128);
        g.nblk = g.tiles_i * (g.tiles_i + 1) / 2;
        b.ns = g.nblk;
        b.s_full = b.ns;
      }
    }
    if (tail_r > 0 && bk == nemit - 1) {
      // the trailing region of this launch is exactly the corner: the tail role replaces its
      // trailing tiles / ragged rows
      b.ns = b.s_full = b.nstrip = 0;
      b.nrag = 0;
      b.ntail = 1;
      b.tail_r = tail_r;
      b.tail_o = cb + CH_NB;
      b.tail_R = (int)(n - b.tail_o);
      b.tail_k0 = bk > 0 ? cb - CH_NB : 0;
      b.tail_K = (int)(b.tail_o - b.tail_k0);
    }
#ifdef IPM_ROLE_TRACE
    {
      static const int tb = [] { const char* e = getenv("IPM_TRACE_BLOCK"); return e ? atoi(e) : -1; }();
      b.trace = bk == tb;
    }
#endif
    b.nra = (int)cdiv(std::max<int64_t>(n - cb - b.wa, 0), PF_RB);
    b.nrb = b.wbw > 0 ? (int)cdiv(std::max<int64_t>(n - cb - wb, 0), PF_RB) : 0;
    {
      const int T = (int)cdiv(b.wbw, 32);
      b.nnf = T * (T + 1) / 2;
    }
    // a plain launch whose trailing tiles can all run the lazy-C loop keeps them whole: the lazy
    // kernel gains more than the K-halves of the last round (r3: 6.20 -> 6.12-6.16 ms at n = 8192)
    static const bool fasts_on = [] { const char* e = getenv("IPM_FASTS"); return !(e && e[0] == '0'); }();
    // (LAZY 2: the block pairs' K = 512 tiles, strips included)
    const bool lazy_cand = lazy_on && fasts_on && vec && (b.s.ni % 128) == 0 &&
                           ((b.s.K == CH_NB && b.nstrip == 0) || (lazy2_on && b.s.K == 2 * CH_NB));
    const bool split_here = split_on && !lazy_cand;
    if (b.s_full > 0 && split_here) {
      // the planner's split count (cached per size and block: it depends on nothing else)
      static std::mutex mu;
      static std::map<std::tuple<int64_t, int64_t, int>, std::vector<int64_t>> cache;
      const int nchd_h = b.wbw > 0 ? (b.wbw + PF_RB - 1) / PF_RB : 0;
      const double tc = b.s.K > CH_NB ? 1.6 : 1.0, lac = Kla > CH_NB ? 1.6 : 0.8;
      const int64_t nra_h = b.nra - nchd_h;
      int64_t q = 0;
      {
        std::lock_guard<std::mutex> lk(mu);
        auto& v = cache[{n, ncols, (lazy_on ? 4 : 0) | (lazy2_on ? 8 : 0) | (vec ? 16 : 0)}];
        if ((int64_t)v.size() < nblocks) v.assign(nblocks, -1);
        if (v[bk] < 0) {
          v[bk] = plan_split(b.nla, nchd_h, b.nnf, b.wbw > 0, b.nrag, b.s_full, nra_h + b.nrb, potrf_split_cap(n),
                             tc, b.nstrip, lac);
          static const bool dbg = getenv("IPM_SPLIT_DEBUG") != nullptr;
          if (dbg)
            fprintf(stderr, "potrf n=%ld block %ld: %ld trailing tiles, split %ld\n", (long)n, (long)bk, (long)b.ns,
                    (long)v[bk]);
        }
        q = v[bk];
      }
      b.s_full -= q;
      b.ns = b.nstrip + b.s_full + 2 * q;
      b.sscr = ws + potrf_split_scratch_off(n);
      b.sflag = b.ctl + block_ctl_words(n) - potrf_split_cap(n);
    }
    BlockLaunch L;
    L.grid = b.nla + 1 + b.nra + b.nnf + (b.wbw > 0 ? 1 + b.nrb : 0) + b.nrag + b.ns + b.ntail;
    // all trailing tiles full (rows a multiple of 128 once the ragged rows are split off) -> the
    // branch-free tile loop (IPM_FASTS=0: never)
    const bool fasts = fasts_on && b.ns > 0 && (b.s.ni % 128) == 0 && (b.s.K % 32) == 0;
    // (r3 A/B, two pairs: 6.48 / 6.52 -> 6.41 / 6.44 ms at the bordered n = 8193; IPM_LAZYC=0: off)
    const bool lazy = lazy_on && fasts && b.s.K == CH_NB && b.nstrip == 0 && b.s_full == b.ns;
    const bool lazy2 = lazy2_on && fasts && b.s.K == 2 * CH_NB && b.nstrip + b.s_full == b.ns &&
                       (b.nstrip == 0 || b.s2.K == 2 * CH_NB) && (b.nrag == 0 || b.rag_K <= 2 * CH_NB);
    L.inst = (vec && lazy) ? 0 : (vec && lazy2) ? 1 : (vec && fasts) ? 2 : vec ? 3 : 4;
    L.b = b;
    out.push_back(L);
  }
}

static void launch_block(hipStream_t st, const BlockLaunch& L) {
  const dim3 g((unsigned)L.grid), t(256);
  switch (L.inst) {
    case 0: hipLaunchKernelGGL((k_potrf_block<true, true, 1>), g, t, 0, st, L.b); break;
    case 1: hipLaunchKernelGGL((k_potrf_block<true, true, 2>), g, t, 0, st, L.b); break;
    case 2: hipLaunchKernelGGL((k_potrf_block<true, true>), g, t, 0, st, L.b); break;
    case 3: hipLaunchKernelGGL((k_potrf_block<true, false>), g, t, 0, st, L.b); break;
    default: hipLaunchKernelGGL((k_potrf_block<false, false>), g, t, 0, st, L.b); break;
  }
}

void potrf_lower_fused(hipStream_t st, int64_t n, double* A, int64_t lda, int* info, double* ws, int64_t ncols,
                       const BorderJob* border) {
  if (ncols < 0 || ncols > n) ncols = n;
  if (border && ncols <= 0) border_rhs(st, border->N, border->H, border->ldh, border->g, border->scale);
  if (ncols <= 0) {
    hipMemsetAsync(info, 0, sizeof(int), st);
    return;
  }
  thread_local std::vector<BlockLaunch> plan;
  potrf_plan(n, A, lda, info, ws, ncols, plan);
  // info, then word 0..7: the "previous launch" of launch 0 (never failed); then cw words per launch
  unsigned* ctl0 = reinterpret_cast<unsigned*>(ws + 2 * PANEL_WS);
  if (border) {
    const int64_t nz = 8 + (int64_t)plan.size() * block_ctl_words(n), tot = 1 + nz + border->N + 1;
    hipLaunchKernelGGL(k_zero2_border, dim3((unsigned)cdiv(tot, 256)), dim3(256), 0, st, reinterpret_cast<unsigned*>(info),
                       (int64_t)1, ctl0, nz, *border);
  } else {
    zero2(st, info, 1, ctl0, 8 + (int64_t)plan.size() * block_ctl_words(n));
  }
  for (const BlockLaunch& L : plan) launch_block(st, L);
}

static int num_cus() {
  static int ncu = -1;
  if (ncu < 0) {
    int dev = 0, v = 0;
    hipGetDevice(&dev);
    ncu = (hipDeviceGetAttribute(&v, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && v > 0) ? v : 256;
  }
  return ncu;
}
#ifdef IPM_ROLE_TRACE
extern "C" int ipm_debug_diag_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ipm_stamps), sizeof(unsigned long long) * 128);
}
extern "C" int ipm_debug_fold_trace(unsigned long long* out) {
#ifdef IPM_ROLE_TRACE
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ipm_fold_trace), sizeof(unsigned long long) * 32 * 12, 0,
                                  hipMemcpyDeviceToHost);
#else
  (void)out;
  return -1;
#endif
}
extern "C" int ipm_debug_role_trace(unsigned long long* out, int n_wg) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ipm_role_trace), sizeof(unsigned long long) * 4 *
                                                                       std::min(n_wg, 8192));
}
#endif

void potrf_lower(hipStream_t st, int64_t n, double* A, int64_t lda, int* info, double* ws) {
  potrf_lower_fused(st, n, A, lda, info, ws);
}

// =====================================================================================
// Triangular solves, L column-major lower, B row-major (n x nrhs).
// One launch per 64-row block: every workgroup redundantly solves the diagonal block
// (from the fully updated B block), workgroup 0 writes it, the others apply it to their
// 64-row chunk of the remaining rows.
// =====================================================================================
constexpr int TS_B = 64;
constexpr int TS_LD = TS_B + 1;
constexpr int TS_R = 8;   // right-hand sides per workgroup pass

// forward: L y = b.  rows below the block are updated: B[i] -= sum_j L[i][j] Y[j]
__global__ __launch_bounds__(256) void k_trsm_fwd_block(int64_t n, int64_t nrhs, int64_t j0, int bs,
                                                        const double* __restrict__ L, int64_t ldl,
                                                        double* __restrict__ B, int64_t ldb,
                                                        double* __restrict__ Y) {
  __shared__ double sL[TS_B * TS_LD];
  __shared__ double sY[TS_B * TS_R];
  __shared__ double sT[TS_B * TS_LD];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < bs * bs; idx += 256) {
    const int j = idx / bs, i = idx % bs;
    sL[i * TS_LD + j] = (i >= j) ? L[(j0 + j) * ldl + j0 + i] : 0.0;
  }
  const int64_t r0 = j0 + bs + (int64_t)(blockIdx.x - 1) * TS_B;
  const int rows = blockIdx.x == 0 ? 0 : (int)max((int64_t)0, min((int64_t)TS_B, n - r0));
  for (int idx = tid; idx < rows * bs; idx += 256) {
    const int j = idx / rows, r = idx % rows;
    sT[r * TS_LD + j] = L[(j0 + j) * ldl + r0 + r];
  }
  for (int64_t c0 = 0; c0 < nrhs; c0 += TS_R) {
    const int nc = (int)min((int64_t)TS_R, nrhs - c0);
    __syncthreads();
    for (int idx = tid; idx < bs * nc; idx += 256) {
      const int i = idx / nc, c = idx % nc;
      sY[i * TS_R + c] = B[(j0 + i) * ldb + c0 + c];
    }
    __syncthreads();
    // forward substitution, thread (i, c): i = tid % 64 rows, c = tid / 64 (4 groups)
    {
      const int i = tid & 63, cg = tid >> 6;
      for (int j = 0; j < bs; ++j) {
        if (i == j)
          for (int c = cg; c < nc; c += 4) sY[j * TS_R + c] /= sL[j * TS_LD + j];
        __syncthreads();
        if (i > j && i < bs)
          for (int c = cg; c < nc; c += 4) sY[i * TS_R + c] -= sL[i * TS_LD + j] * sY[j * TS_R + c];
        __syncthreads();
      }
    }
    if (blockIdx.x == 0) {
      for (int idx = tid; idx < bs * nc; idx += 256) {
        const int i = idx / nc, c = idx % nc;
        Y[(j0 + i) * ldb + c0 + c] = sY[i * TS_R + c];
      }
    } else {
      for (int idx = tid; idx < rows * nc; idx += 256) {
        const int r = idx / nc, c = idx % nc;
        double acc = 0.0;
        for (int j = 0; j < bs; ++j) acc = fma(sT[r * TS_LD + j], sY[j * TS_R + c], acc);
        B[(r0 + r) * ldb + c0 + c] -= acc;
      }
    }
  }
}

// backward: L^T x = y.  rows above the block are updated: B[i] -= sum_{j in block} L[j][i] X[j]
__global__ __launch_bounds__(256) void k_trsm_bwd_block(int64_t n, int64_t nrhs, int64_t j0, int bs,
                                                        const double* __restrict__ L, int64_t ldl,
                                                        double* __restrict__ B, int64_t ldb,
                                                        double* __restrict__ Y) {
  __shared__ double sL[TS_B * TS_LD];
  __shared__ double sY[TS_B * TS_R];
  __shared__ double sT[TS_B * TS_LD];
  const int tid = threadIdx.x;
  for (int idx = tid; idx < bs * bs; idx += 256) {
    const int j = idx / bs, i = idx % bs;
    sL[i * TS_LD + j] = (i >= j) ? L[(j0 + j) * ldl + j0 + i] : 0.0;
  }
  // columns above: [c0, c0 + 64) with c0 = (g-1)*64 < j0; tile sT[c][j] = L[j0 + j][c0 + c]
  const int64_t cbeg = (int64_t)(blockIdx.x - 1) * TS_B;
  const int cols = blockIdx.x == 0 ? 0 : (int)max((int64_t)0, min((int64_t)TS_B, j0 - cbeg));
  for (int idx = tid; idx < cols * bs; idx += 256) {
    const int c = idx / bs, j = idx % bs;
    sT[c * TS_LD + j] = L[(cbeg + c) * ldl + j0 + j];
  }
  for (int64_t q0 = 0; q0 < nrhs; q0 += TS_R) {
    const int nc = (int)min((int64_t)TS_R, nrhs - q0);
    __syncthreads();
    for (int idx = tid; idx < bs * nc; idx += 256) {
      const int i = idx / nc, c = idx % nc;
      sY[i * TS_R + c] = B[(j0 + i) * ldb + q0 + c];
    }
    __syncthreads();
    {
      const int i = tid & 63, cg = tid >> 6;
      for (int j = bs - 1; j >= 0; --j) {
        if (i == j)
          for (int c = cg; c < nc; c += 4) sY[j * TS_R + c] /= sL[j * TS_LD + j];
        __syncthreads();
        if (i < j)
          for (int c = cg; c < nc; c += 4) sY[i * TS_R + c] -= sL[j * TS_LD + i] * sY[j * TS_R + c];
        __syncthreads();
      }
    }
    if (blockIdx.x == 0) {
      for (int idx = tid; idx < bs * nc; idx += 256) {
        const int i = idx / nc, c = idx % nc;
        Y[(j0 + i) * ldb + q0 + c] = sY[i * TS_R + c];
      }
    } else {
      for (int idx = tid; idx < cols * nc; idx += 256) {
        const int r = idx / nc, c = idx % nc;
        double acc = 0.0;
        for (int j = 0; j < bs; ++j) acc = fma(sT[r * TS_LD + j], sY[j * TS_R + c], acc);
        B[(cbeg + r) * ldb + q0 + c] -= acc;
      }
    }
  }
}

// B is consumed (rows are updated in place); the solution is written to Y (n x nrhs, ldb).
void trsm_lower_fwd(hipStream_t st, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B,
                    int64_t ldb, double* Y) {
  for (int64_t j0 = 0; j0 < n; j0 += TS_B) {
    const int bs = (int)std::min<int64_t>(TS_B, n - j0);
    const int64_t below = n - j0 - bs;
    dim3 g(1 + cdiv(below, TS_B));
    hipLaunchKernelGGL(k_trsm_fwd_block, g, dim3(256), 0, st, n, nrhs, j0, bs, L, ldl, B, ldb, Y);
  }
}

void trsm_lower_bwd(hipStream_t st, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B,
                    int64_t ldb, double* Y) {
  const int64_t nblk = cdiv(n, TS_B);
  for (int64_t blk = nblk - 1; blk >= 0; --blk) {
    const int64_t j0 = blk * TS_B;
    const int bs = (int)std::min<int64_t>(TS_B, n - j0);
    dim3 g(1 + cdiv(j0, TS_B));
    hipLaunchKernelGGL(k_trsm_bwd_block, g, dim3(256), 0, st, n, nrhs, j0, bs, L, ldl, B, ldb, Y);
  }
}

// =====================================================================================
// Single right-hand side (the Newton step of NewtonSolver.py:287-299 / 303-313): each
// direction is ONE persistent launch.  The solve is HBM-bound (L is read once, 8 n^2/2
// bytes); its critical path is the chain of 64x64 diagonal-block solves, so everything
// else is taken off that chain:
//   * workgroups draw block tickets in solve order (atomic ctl[0]); the owner of block B
//     streams the off-diagonal tiles of its block row (fwd) / block column (bwd) into
//     registers one tile AHEAD of the published solutions it multiplies them with,
//   * the diagonal block is staged in LDS and its reciprocal pivots computed while the
//     workgroup waits, and the 64-step substitution runs in one wave out of registers
//     (readlane broadcasts, no barriers),
//   * the 64 results are published with agent-scope (sc1) stores by that one wave, then
//     s_waitcnt vmcnt(0), then the progress word ctl[1] = ticket + 1 (sc1).  Consumers poll
//     the progress word and read the published values with sc1 loads only -- the hand-off
//     form of MI355X_MICROARCH.md "Valid forms" (no acquire fence on the chain).
// A workgroup only ever waits on blocks with SMALLER tickets, which are held by running
// workgroups, so any grid size makes progress; every workgroup exits when tickets run out.
// Blocks are published in ticket order, so "progress > t" means tickets 0..t are solved.
// =====================================================================================
constexpr int TV_B = 64;

__device__ __forceinline__ double bcast_d(double v, int l) {   // l wave-uniform
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}

// FWD: solve L y = b.   !FWD: solve L^T y = b.   L column-major lower (ldl); y must not alias b.
template <bool FWD>
__global__ __launch_bounds__(256) void k_trsv_chain(int64_t n, int nblk, const double* __restrict__ L,
                                                    int64_t ldl, const double* __restrict__ b, int64_t bstride,
                                                    double* y, unsigned* ctl) {
  __shared__ double sL[TV_B * (TV_B + 1)];        // diagonal block, column-major, padded
  __shared__ double sdinv[TV_B];
  __shared__ double sacc[TV_B * (TV_B + 1)];      // cross-wave / cross-lane partial sums
  __shared__ int sticket;
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  for (;;) {
    if (tid == 0) sticket = (int)atomicAdd(&ctl[0], 1u);
    __syncthreads();
    const int t = sticket;
    __syncthreads();
    if (t >= nblk) break;
    const int B = FWD ? t : nblk - 1 - t;                 // block this workgroup solves
    const int64_t r0 = (int64_t)B * TV_B;
    const int rows = (int)min((int64_t)TV_B, n - r0);
    const int ntile = t;                                  // tiles from already-solved blocks
    // ---- off-diagonal tile t' (ticket order): 16 columns per wave, lane = tile row
    //   FWD: tile L[B, J] with J = t'            -> rows r0.., columns J*64 + w*16 + jj
    //   BWD: tile L[K, B] with K = nblk-1-t'     -> rows K*64.., columns r0 + w*16 + jj
    auto load_tile = [&](int tp, double (&dst)[16]) {
      if (FWD) {
        const double* base = L + ((int64_t)tp * TV_B + w * 16) * ldl + r0 + lane;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) dst[jj] = lane < rows ? base[jj * ldl] : 0.0;
      } else {
        const int64_t k0 = (int64_t)(nblk - 1 - tp) * TV_B;
        const int krows = (int)min((int64_t)TV_B, n - k0);
        const double* base = L + (r0 + w * 16) * ldl + k0 + lane;
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) dst[jj] = lane < krows ? base[jj * ldl] : 0.0;
      }
    };
    double cur[16], nxt[16];
    if (ntile > 0) load_tile(0, cur);
    // stage the diagonal block (lower part) and the reciprocal pivots while tiles stream in
    for (int idx = tid; idx < TV_B * TV_B; idx += 256) {
      const int j = idx >> 6, i = idx & 63;
      sL[j * (TV_B + 1) + i] = (i < rows && j < rows && i >= j) ? L[(r0 + j) * ldl + r0 + i] : 0.0;
    }
    __syncthreads();
    if (tid < TV_B) sdinv[tid] = tid < rows ? 1.0 / sL[tid * (TV_B + 1) + tid] : 0.0;
    double accf = 0.0;
    double accb[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) accb[jj] = 0.0;
    unsigned known = 0;
    for (int tp = 0; tp < ntile; ++tp) {
      // poll first, then issue the next tile's loads, then wait only for the poll
      if (known <= (unsigned)tp) known = ld_ctl(&ctl[1]);
      if (tp + 1 < ntile) load_tile(tp + 1, nxt);
      while (known <= (unsigned)tp) {
        __builtin_amdgcn_s_sleep(1);
        known = ld_ctl(&ctl[1]);
      }
      if (FWD) {
        // y_J of this wave's 16 columns: wave-uniform sc1 loads (one request each)
        const double* yj = y + (int64_t)tp * TV_B + w * 16;
        double v[16];
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) v[jj] = ld_sc1(yj + jj);
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) accf = fma(cur[jj], v[jj], accf);
      } else {
        const int64_t k0 = (int64_t)(nblk - 1 - tp) * TV_B;
        const double v = (k0 + lane < n) ? ld_sc1(y + k0 + lane) : 0.0;   // x_K, lane = row
#pragma unroll
        for (int jj = 0; jj < 16; ++jj) accb[jj] = fma(cur[jj], v, accb[jj]);
      }
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) cur[jj] = nxt[jj];
    }
    // ---- reduce the partial sums of the 4 waves (fixed order: deterministic)
    if (FWD) {
      sacc[w * (TV_B + 1) + lane] = accf;
    } else {
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) sacc[(w * 16 + jj) * (TV_B + 1) + lane] = accb[jj];
    }
    __syncthreads();
    if (w == 0) {
      double s;
      if (FWD) {
        s = (sacc[lane] + sacc[(TV_B + 1) + lane]) + (sacc[2 * (TV_B + 1) + lane] + sacc[3 * (TV_B + 1) + lane]);
      } else {
        s = 0.0;
        for (int l = 0; l < TV_B; ++l) s += sacc[lane * (TV_B + 1) + l];
      }
      double r = lane < rows ? b[(r0 + lane) * bstride] - s : 0.0;
      const double dinv = sdinv[lane];
      // Substitution out of registers.  lv holds the STRICTLY triangular part of the lane's
      // row (fwd) / column (bwd), so step j leaves lanes <= j (fwd) / >= j (bwd) untouched and
      // lane j's final value is y_j = r_j * dinv_j -- no per-step lane masks on the chain.
      double lv[TV_B];
      if (FWD) {
        // lane i: L[i][j] (j < i) at sL[j*65 + i]
#pragma unroll
        for (int j = 0; j < TV_B; ++j) lv[j] = lane > j ? sL[j * (TV_B + 1) + lane] : 0.0;
#pragma unroll
        for (int j = 0; j < TV_B; ++j) r = fma(-lv[j], bcast_d(r * dinv, j), r);
      } else {
        // lane k: L[j][k] (j > k) at sL[k*65 + j];  L^T x = r solved for j = 63 .. 0
#pragma unroll
        for (int j = 0; j < TV_B; ++j) lv[j] = lane < j ? sL[lane * (TV_B + 1) + j] : 0.0;
#pragma unroll
        for (int j = TV_B - 1; j >= 0; --j) r = fma(-lv[j], bcast_d(r * dinv, j), r);
      }
      r = r * dinv;
      if (lane < rows) st_sc1(y + r0 + lane, r);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      if (lane == 0) __hip_atomic_store(&ctl[1], (unsigned)(t + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
  }
}

// -------------------------------------------------------------------------------------
// Backward solve L^T x = b in 128-row blocks (the Newton step's second cho_solve half,
// NewtonSolver.py:303-313; the first half rides inside the Cholesky as the bordered row).
// Half the chain steps of the 64-row kernel, and each step is two small matrix-vector products
// instead of a 64-step substitution: the owner of block B (ticket t = nblk-1-B, one workgroup of
// 8 waves) computes, OFF the chain,
//   * X_B = L_BB^-T (128 x 128, upper) by the panel kernels' 8-step MFMA block substitution
//     X L_BB^T = I with inverted 16 x 16 diagonal blocks (wave w: rows 16w .. 16w+15),
//   * pre = sum_{K >= B+2} L_KB^T x_K, streamed as those blocks are published,
// and loads the tile L_{B+1,B} into registers.  The chain step is then
//   rhs = b_B - pre - L_{B+1,B}^T x_{B+1};   x_B = X_B rhs
// with thread (c, q) (c = column, q = quarter of the 128 k-indices) holding L_{B+1,B}[32q.., c]
// in registers and X_B in LDS.  Hand-off as k_trsv_chain (sc1 stores, vmcnt(0), progress
// word; consumers poll and read with sc1 loads).
// -------------------------------------------------------------------------------------
constexpr int TB2 = 128;
// X_B = L_BB^-T for every 128-row diagonal block, one workgroup (8 waves) per block: the 8-step
// MFMA block substitution X L_BB^T = I of the panel kernels' row role (wave w: rows 16w ..
// 16w+15; X_J = 0 for J < w) with inverted 16 x 16 diagonal blocks.  Xws: nblk blocks of
// 128 x 128, X[c][r] at c * 128 + r.  Identity beyond the last row.
struct TrinvSmem {
  double sD[36 * 256];
  double sDinv[8 * 256];
  double srinv[8 * 16];
};
// (y, ctl non-null: also resets the backward solve's state, saving two memset launches per solve:
// y's block B to the pending pattern, and the solve's two control words by workgroup 0)
__global__ __launch_bounds__(512, 1) void k_trinv128(int64_t n, const double* __restrict__ L, int64_t ldl,
                                                     double* __restrict__ Xws, double* __restrict__ y,
                                                     unsigned* __restrict__ ctl) {
  __shared__ TrinvSmem sm;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int fr = lane & 15, fk = lane >> 4;
  const int B = blockIdx.x;
  const int64_t r0 = (int64_t)B * TB2;
  const int rows = (int)min((int64_t)TB2, n - r0);
  if (y && tid < rows) y[r0 + tid] = __longlong_as_double(-1LL);   // TRSV_PENDING
  if (ctl && B == 0 && tid < 2) ctl[tid] = 0u;
  for (int idx = tid; idx < 36 * 256; idx += 512) {
    const int blk = idx >> 8, e = idx & 255, rr = e & 15, cc = e >> 4;
    int I = 0;
    while ((I + 1) * (I + 2) / 2 <= blk) ++I;
    const int J = blk - I * (I + 1) / 2;
    const int i = I * 16 + rr, j = J * 16 + cc;
    double v;
    if (i < rows && j < rows) v = (i >= j) ? L[(r0 + j) * ldl + r0 + i] : 0.0;
    else v = (i == j) ? 1.0 : 0.0;
    sm.sD[idx] = v;
  }
  __syncthreads();
  if (lane < 16) sm.srinv[wv * 16 + lane] = 1.0 / sm.sD[bidx(wv, wv) * 256 + lane * 16 + lane];
  __syncthreads();
  tri_inverse16(&sm.sD[bidx(wv, wv) * 256], &sm.srinv[wv * 16], &sm.sDinv[wv * 256], lane, false);
  __syncthreads();
  dbl4 x[8];
#pragma unroll
  for (int J = 0; J < 8; ++J) {
    x[J] = dbl4{0.0, 0.0, 0.0, 0.0};
    if (J < wv) continue;
    dbl4 acc;
#pragma unroll
    for (int r = 0; r < 4; ++r) acc[r] = (J == wv && fr == fk + 4 * r) ? 1.0 : 0.0;   // identity block
#pragma unroll
    for (int P = 0; P < J; ++P) {
      if (P < wv) continue;
      const double* lb = &sm.sD[bidx(J, P) * 256 + fk * 16 + fr];
      double av[4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) av[s4] = -lb[64 * s4];
#pragma unroll
      for (int s4 = 0; s4 < 4; ++s4) acc = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], x[P][s4], acc, 0, 0, 0);
    }
    const double* ib = &sm.sDinv[J * 256 + fk * 16 + fr];
    dbl4 xj = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int s4 = 0; s4 < 4; ++s4) xj = __builtin_amdgcn_mfma_f64_16x16x4f64(ib[64 * s4], acc[s4], xj, 0, 0, 0);
    x[J] = xj;
  }
  // lane holds X[16w + fr][16J + fk + 4r]
  double* xo = Xws + (int64_t)B * TB2 * TB2;
#pragma unroll
  for (int J = 0; J < 8; ++J)
#pragma unroll
    for (int r = 0; r < 4; ++r) xo[(16 * wv + fr) * TB2 + 16 * J + fk + 4 * r] = x[J][r];
}

// -------------------------------------------------------------------------------------
// Backward solve L^T x = b in 128-row blocks (the Newton step's second cho_solve half,
// NewtonSolver.py:303-313; the first half rides inside the Cholesky as the bordered row).
// Half the chain steps of the 64-row kernel, and each step is two matrix-vector products
// instead of a 64-step substitution.  The owner of block B (ticket t = nblk-1-B, one workgroup
// of 8 waves) loads X_B = L_BB^-T (k_trinv128) into LDS, streams
//   pre = sum_{K >= B+2} L_KB^T x_K
// as those blocks are published, and holds the tile L_{B+1,B} in registers (thread (c, q): column
// c, k-indices 32q .. 32q+31), all off the chain.  The chain step is then
//   rhs = b_B - pre - L_{B+1,B}^T x_{B+1};   x_B = X_B rhs.
// Hand-off: sc1 stores of the x block; every consumer polls the x values it needs with sc1 loads
// (y starts as TRSV_PENDING), the chain step and (r6) the pre sum alike.  The progress word is still
// published (monotonic) but no longer waited on.  r6 hand-off lab (tools/handoff_lab.hip): one
// store -> poll hop costs ~0.6 us, on one XCD or across XCDs alike.
// -------------------------------------------------------------------------------------
constexpr long long TRSV_PENDING = -1LL;
#ifdef IPM_ROLE_TRACE
// backward-solve stamps of the last solve (trace builds): per ticket [0] pre sum done, [1] x_{B+1}
// polled, [2] x_B stored (s_memrealtime)
__device__ unsigned long long ipm_trsv_trace[512 * 4];
extern "C" int ipm_debug_trsv_trace(unsigned long long* out, int n) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(ipm_trsv_trace), sizeof(unsigned long long) * 4 * std::min(n, 512));
}
#define TRSV_STAMP(k) do { if (tid == 0 && t < 512) ipm_trsv_trace[4 * t + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define TRSV_STAMP(k) do {} while (0)
#endif   // 0xFFFF...F: y's content before its block is solved
struct Trsv128Smem {
  double sX[TB2 * (TB2 + 1)];   // X_B, X[c][r] at r * 129 + c
  double sx[TB2];               // x_{B+1}
  double sv[TB2];               // rhs
  double spart[4][TB2];         // per-quarter partial sums
  double spre[TB2];             // pre
};

__global__ __launch_bounds__(512, 1) void k_trsv_bwd128(int64_t n, int nblk, const double* __restrict__ L,
                                                        int64_t ldl, const double* __restrict__ b, int64_t bstride,
                                                        const double* __restrict__ Xws, double* y, unsigned* ctl,
                                                        unsigned* err, int delay_ticket) {
  __shared__ Trsv128Smem sm;
  __shared__ int sticket;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;   // 8 waves
  const int c = tid & 127, q = tid >> 7;                          // critical layout
  for (;;) {
    if (tid == 0) sticket = (int)atomicAdd(&ctl[0], 1u);
    __syncthreads();
    const int t = sticket;
    __syncthreads();
    if (t >= nblk) break;
    const int B = nblk - 1 - t;
    const int64_t r0 = (int64_t)B * TB2;
    const int rows = (int)min((int64_t)TB2, n - r0);
    {
      const double* xs = Xws + (int64_t)B * TB2 * TB2;
      for (int idx = tid; idx < TB2 * TB2; idx += 512) {
        const int cc = idx >> 7, r = idx & 127;   // X[cc][r]
        sm.sX[r * (TB2 + 1) + cc] = xs[idx];
      }
    }
    const double bval = (q == 0 && c < rows) ? b[(r0 + c) * bstride] : 0.0;
    // the tile L_{B+1,B} (rows of block B+1, columns of B): loaded first, it is needed right
    // after the streaming below
    double lt[32];
    {
      const int64_t k0 = r0 + TB2;
      const int krows = (int)max((int64_t)0, min((int64_t)TB2, n - k0));
#pragma unroll
      for (int k = 0; k < 32; ++k)
        lt[k] = (B + 1 < nblk && c < rows && 32 * q + k < krows) ? L[(r0 + c) * ldl + k0 + 32 * q + k] : 0.0;
    }
    // ---- pre = sum_{K >= B+2} L_KB^T x_K in publication order; thread (lane, wave): rows
    //      2 lane, 2 lane + 1 of each tile, columns 16 w .. 16 w + 15
    double acc[16];
#pragma unroll
    for (int jj = 0; jj < 16; ++jj) acc[jj] = 0.0;
    // (r6: each lane polls its two x values themselves -- y starts as TRSV_PENDING -- instead of
    // waiting for the progress word of their ticket: the word is published after the y store, its
    // wait, a barrier and an atomic, and the pre sum's last term (x_{B+2}) sat on the chain behind
    // that extra round trip.  The same fma sequence: bitwise the same x.)
    bool released = false;   // a poll ran out its bound: x is garbage, the error word says so
#pragma nounroll
    for (int tp = 0; tp + 1 < t; ++tp) {
      const int64_t k0 = (int64_t)(nblk - 1 - tp) * TB2;
      const int krows = (int)min((int64_t)TB2, n - k0);
      const int kr = 2 * lane;
      double tv0[16], tv1[16];
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) {
        const int cc = 16 * wv + jj;
        const double* src = L + (r0 + cc) * ldl + k0 + kr;
        tv0[jj] = (cc < rows && kr < krows) ? src[0] : 0.0;
        tv1[jj] = (cc < rows && kr + 1 < krows) ? src[1] : 0.0;
      }
      double x0 = 0.0, x1 = 0.0;
      auto landed = [&] {
        x0 = kr < krows ? ld_sc1(y + k0 + kr) : 0.0;
        x1 = kr + 1 < krows ? ld_sc1(y + k0 + kr + 1) : 0.0;
        return __double_as_longlong(x0) != TRSV_PENDING && __double_as_longlong(x1) != TRSV_PENDING;
      };
      if (released) {
        landed();
      } else if (!spin_until<1, 1>(nullptr, nullptr, landed)) {
        __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        released = true;
      }
#pragma unroll
      for (int jj = 0; jj < 16; ++jj) acc[jj] = fma(tv1[jj], x1, fma(tv0[jj], x0, acc[jj]));
    }
    // transpose-reduce the 16 column sums over the 64 lanes (17 shuffles): the halving steps over
    // lane bits 5..2 leave each lane one column summed over 16 lanes
    {
      double v8[8], v4[4], v2[2], v1;
      const bool u5 = lane & 32, u4 = lane & 16, u3 = lane & 8, u2 = lane & 4;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const double snd = u5 ? acc[i] : acc[i + 8], kp = u5 ? acc[i + 8] : acc[i];
        v8[i] = kp + __shfl_xor(snd, 32, 64);
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const double snd = u4 ? v8[i] : v8[i + 4], kp = u4 ? v8[i + 4] : v8[i];
        v4[i] = kp + __shfl_xor(snd, 16, 64);
      }
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const double snd = u3 ? v4[i] : v4[i + 2], kp = u3 ? v4[i + 2] : v4[i];
        v2[i] = kp + __shfl_xor(snd, 8, 64);
      }
      {
        const double snd = u2 ? v2[0] : v2[1], kp = u2 ? v2[1] : v2[0];
        v1 = kp + __shfl_xor(snd, 4, 64);
      }
      v1 += __shfl_xor(v1, 2, 64);
      v1 += __shfl_xor(v1, 1, 64);
      const int col = (u5 ? 8 : 0) + (u4 ? 4 : 0) + (u3 ? 2 : 0) + (u2 ? 1 : 0);
      if ((lane & 3) == 0) sm.spre[16 * wv + col] = v1;
    }
    __syncthreads();
    TRSV_STAMP(0);
    // X_B's entries of this thread's second product (X[c][32q + k]) into registers before the chain
    // step (r6: off the chain; the same fma sequence as reading them from LDS inside it)
    double xrg[32];
#pragma unroll
    for (int k = 0; k < 32; ++k) xrg[k] = sm.sX[(32 * q + k) * (TB2 + 1) + c];
    // ---- the chain step
    if (t > 0) {
      const int64_t k0 = r0 + TB2;
      const int krows = (int)min((int64_t)TB2, n - k0);
      // x_{B+1} is polled directly (y starts as the all-ones NaN pattern, which no fp64 arithmetic
      // produces -- b must not hold it either, trsv_lower_t's contract): no progress-word round trip
      // on the chain.  The spin is bounded: a producer that has not published after spin_limit
      // wall-clock bound (s_memrealtime, ipm_spin_ticks[1]) raises the sticky device error word *err (bit 0),
      // which the host reads with the Newton step's readback and turns into IPM_HIP_ERROR -- the step
      // is never used silently.
      if (tid < TB2) {
        double v = 0.0;
        if (tid < krows) {
          if (!spin_until<1, 1>(nullptr, nullptr, [&] {
                v = ld_sc1(y + k0 + tid);
                return __double_as_longlong(v) != TRSV_PENDING;
              }))
            __hip_atomic_fetch_or(err, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        sm.sx[tid] = v;
      }
      __syncthreads();
      TRSV_STAMP(1);
      double p = 0.0, p2 = 0.0;
#pragma unroll
      for (int k = 0; k < 32; k += 2) {
        p = fma(lt[k], sm.sx[32 * q + k], p);
        p2 = fma(lt[k + 1], sm.sx[32 * q + k + 1], p2);
      }
      sm.spart[q][c] = p + p2;
    } else {
      sm.spart[q][c] = 0.0;
    }
    __syncthreads();
    if (q == 0) sm.sv[c] = bval - sm.spre[c] - ((sm.spart[0][c] + sm.spart[1][c]) + (sm.spart[2][c] + sm.spart[3][c]));
    __syncthreads();
    {
      double p = 0.0, p2 = 0.0;
#pragma unroll
      for (int k = 0; k < 32; k += 2) {
        p = fma(xrg[k], sm.sv[32 * q + k], p);
        p2 = fma(xrg[k + 1], sm.sv[32 * q + k + 1], p2);
      }
      // (spart's last readers were the sv line above, before the barrier: no barrier needed here)
      sm.spart[q][c] = p + p2;
    }
    __syncthreads();
    if (delay_ticket <= -2 && t == -2 - delay_ticket) {   // debug knob: a late x store (trips the
      for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(127);   // next ticket's bounded poll)
    }
    if (q == 0 && c < rows)
      st_sc1(y + r0 + c, (sm.spart[0][c] + sm.spart[1][c]) + (sm.spart[2][c] + sm.spart[3][c]));
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    TRSV_STAMP(2);
    // publish "tickets <= t solved": monotonic.  With the data-polled chain a later ticket can finish
    // (it only needs x_{B+1}, which it read from y) before this store lands; a plain store could
    // then move ctl[1] backwards and leave the pre loop above waiting forever.
    if (t == delay_ticket) {   // debug knob: a late publisher (tests the monotonic publish)
      for (int i = 0; i < 2000; ++i) __builtin_amdgcn_s_sleep(127);
    }
    if (tid == 0) __hip_atomic_fetch_max(&ctl[1], (unsigned)(t + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __syncthreads();
  }
}

static void trsv_chain(hipStream_t st, bool fwd, int64_t n, const double* L, int64_t ldl, const double* b,
                       int64_t bstride, double* y, unsigned* ctl) {
  const int nblk = (int)cdiv(n, TV_B);
  const int grid = std::min(nblk, 1024);
  if (fwd)
    hipLaunchKernelGGL(k_trsv_chain<true>, dim3(grid), dim3(256), 0, st, n, nblk, L, ldl, b, bstride, y, ctl);
  else
    hipLaunchKernelGGL(k_trsv_chain<false>, dim3(grid), dim3(256), 0, st, n, nblk, L, ldl, b, bstride, y, ctl);
}

// the chain poll's bound in microseconds of wall clock (a sleep count depends on the
// clock and a descheduled producer); 0 restores the default 1 s
static std::atomic<int> g_trsv_delay_ticket{-1};
void set_trsv_spin_limit(unsigned us) { set_spin_ticks(1, us); }
void set_trsv_publish_delay(int ticket) { g_trsv_delay_ticket.store(ticket); }

// L^T x = b (b read with stride bstride, e.g. the bordered row of a Cholesky factor); ctl: 2 words
void trsv_lower_t(hipStream_t st, int64_t n, const double* L, int64_t ldl, const double* b, int64_t bstride,
                  double* x, unsigned* ctl, double* xinv_ws, unsigned* err) {
  if (n <= 0) return;
  // without the inverse workspace (or IPM_TRSV64=1): the 64-row substitution kernel
  static const bool k64 = [] { const char* e = getenv("IPM_TRSV64"); return e && e[0] == '1'; }();
  if (k64 || !xinv_ws || !err) {
    hipMemsetAsync(ctl, 0, 2 * sizeof(unsigned), st);
    trsv_chain(st, false, n, L, ldl, b, bstride, x, ctl);
    return;
  }
  const int nblk = (int)cdiv(n, TB2);
  // (k_trinv128 also sets x to TRSV_PENDING in every row and zeroes ctl)
  hipLaunchKernelGGL(k_trinv128, dim3(nblk), dim3(512), 0, st, n, L, ldl, xinv_ws, x, ctl);
  const int grid = std::min(nblk, 256);
  hipLaunchKernelGGL(k_trsv_bwd128, dim3(grid), dim3(512), 0, st, n, nblk, L, ldl, b, bstride, xinv_ws, x, ctl,
                     err,
                     g_trsv_delay_ticket.load(std::memory_order_relaxed));
}

// Bordered right-hand side: row N of the (N+1) x (N+1) column-major lower factor input holds
// rhs^T and the corner a huge value, so that the Cholesky factor's row N is (L^-1 rhs)^T -- the
// forward substitution comes out of the factorisation itself (Cholesky of [[H, r], [r^T, c]]).
__global__ void k_border_rhs(int64_t N, double* H, int64_t ldh, const double* g, double scale, double corner) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < N) H[j * ldh + N] = scale * g[j];
  else if (j == N) H[N * ldh + N] = corner;
}
void border_rhs(hipStream_t st, int64_t N, double* H, int64_t ldh, const double* g, double scale) {
  hipLaunchKernelGGL(k_border_rhs, dim3(cdiv(N + 1, 256)), dim3(256), 0, st, N, H, ldh, g, scale, 1e300);
}

// L L^T X = B in place; W: scratch n x nrhs (ldb); ctl: device scratch of 4 words (single
// right-hand side only; may be null, then the blocked multi-RHS path is used)
void potrs_lower(hipStream_t st, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B,
                 int64_t ldb, double* W, unsigned* ctl, double* xinv_ws, unsigned* err) {
  if (n <= 0 || nrhs <= 0) return;
  if (nrhs == 1 && ldb == 1 && ctl) {
    hipMemsetAsync(ctl, 0, 4 * sizeof(unsigned), st);
    trsv_chain(st, true, n, L, ldl, B, 1, W, ctl);
    trsv_lower_t(st, n, L, ldl, W, 1, B, ctl + 2, xinv_ws, err);
    return;
  }
  trsm_lower_fwd(st, n, nrhs, L, ldl, B, ldb, W);
  trsm_lower_bwd(st, n, nrhs, L, ldl, W, ldb, B);
}

// ---- many right-hand sides: L L^T X = B in 128-row blocks on fp64 MFMA GEMMs (the Lasso's
// cho_solve(., I), LassoSolver.py:178-189; the per-column substitution kernels above take seconds
// at n = 4096 with n right-hand sides).  B row-major n x nrhs.  With Xs_j = L_jj^-T (k_trinv128,
// row-major 128 x 128: as a k-major operand it is L_jj^-1) and its transpose XsT_j (= L_jj^-T as a
// k-major operand):
//   forward  Y_j = L_jj^-1 B_j;            B_i -= L_ij Y_j        (i > j; L columns are k-major)
//   backward X_j = L_jj^-T Y_j;            B_i -= L_ji^T X_j      (i < j; rows of L: the row-major
//                                                                   copy Lr, k-major)
// Every product is C(s, r) = sum_k X[k][s] Y[k][r] of the MFMA tile with C = the row-major block.
__global__ void k_block_transpose128(int64_t nblk, const double* __restrict__ in, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= nblk * 16384) return;
  const int64_t b = e >> 14, q = e & 16383, r = q >> 7, c = q & 127;
  out[(b << 14) + c * 128 + r] = in[(b << 14) + r * 128 + c];
}
__global__ void k_copy_rows(int64_t rows, int64_t cols, const double* __restrict__ in, int64_t ldi,
                            double* __restrict__ out, int64_t ldo) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= rows * cols) return;
  const int64_t r = e / cols, c = e - r * cols;
  out[r * ldo + c] = in[r * ldi + c];
}
// workspace: the inverted diagonal blocks and their transposes, ONE 128-row panel of L transposed
// for the backward GEMMs (128 n doubles, not a transposed copy of all of L), the diag staging
int64_t potrs_blocked_ws_doubles(int64_t n, int64_t nrhs) {
  const int64_t nblk = cdiv(n, 128);
  return 2 * nblk * 16384 + 128 * n + 128 * nrhs + 64;
}
void potrs_blocked(hipStream_t st, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B, int64_t ldb,
                   double* ws) {
  if (n <= 0 || nrhs <= 0) return;
  const int64_t nblk = cdiv(n, 128);
  double* Xs = ws;
  double* XsT = Xs + nblk * 16384;
  double* Lp = XsT + nblk * 16384;   // Lp[k * n + c] = L(j0 + k, c), c < j0: block row j, transposed
  double* T = Lp + 128 * n;
  hipLaunchKernelGGL(k_trinv128, dim3((unsigned)nblk), dim3(512), 0, st, n, L, ldl, Xs, nullptr, nullptr);
  hipLaunchKernelGGL(k_block_transpose128, dim3((unsigned)cdiv(nblk * 16384, 256)), dim3(256), 0, st, nblk, Xs, XsT);
  auto gemm = [&](int64_t ni, int64_t nj, int64_t K, const double* X, int64_t ldx, const double* Y, int64_t ldy,
                  double* C, int64_t ldc, bool sub) {
    if (ni <= 0 || nj <= 0 || K <= 0) return;
    GemmArgs g;
    g.ni = ni;
    g.nj = nj;
    g.K = K;
    g.X = X;
    g.ldx = ldx;
    g.Y = Y;
    g.ldy = ldy;
    g.C = C;
    g.ldc = ldc;
    g.sub = sub ? 1 : 0;
    mfma_gemm_launch(st, g);
  };
  auto diag = [&](int64_t j, const double* Yblk) {   // B_j <- inv-block * B_j (through T)
    const int64_t j0 = j * 128, bj = std::min<int64_t>(128, n - j0);
    gemm(nrhs, bj, bj, B + j0 * ldb, ldb, Yblk, 128, T, nrhs, false);
    hipLaunchKernelGGL(k_copy_rows, dim3((unsigned)cdiv(bj * nrhs, 256)), dim3(256), 0, st, bj, nrhs, T, nrhs,
                       B + j0 * ldb, ldb);
  };
  for (int64_t j = 0; j < nblk; ++j) {
    const int64_t j0 = j * 128, j1 = std::min<int64_t>(n, j0 + 128);
    diag(j, Xs + j * 16384);
    gemm(nrhs, n - j1, j1 - j0, B + j0 * ldb, ldb, L + j0 * ldl + j1, ldl, B + j1 * ldb, ldb, true);
  }
  for (int64_t j = nblk - 1; j >= 0; --j) {
    const int64_t j0 = j * 128, j1 = std::min<int64_t>(n, j0 + 128);
    diag(j, XsT + j * 16384);
    if (j0 > 0) {
      transpose(st, j0, j1 - j0, L + j0, ldl, Lp, n);   // (the panel the GEMM below reads)
      gemm(nrhs, j0, j1 - j0, B + j0 * ldb, ldb, Lp, n, B, ldb, true);
    }
  }
}

// ---- LU with partial pivoting (np.linalg.solve; the Cholesky fallback, Q9), column-major.
// Blocked right-looking: panels of LU_NB columns are factored column by column (pivot search,
// swap and scale in one workgroup; the rank-1 update restricted to the panel), then the panel's
// row swaps go to the other columns (k_laswp), U12 = L11^-1 A12 (k_lu_trsm) and the trailing
// matrix takes A22 -= L21 U12 as ONE fp64-MFMA GEMM (the trailing update of the unblocked form
// re-streamed the whole matrix once per column).  Pivot choice = LAPACK's (first index of the
// largest |a|).  An exactly zero pivot column is skipped (piv = -1 - k, its L column zeroed so the
// blocked updates see no contribution), like the unblocked form: getrs then gives that component 0.
constexpr int LU_NB = 64;

__global__ __launch_bounds__(1024) void k_lu_pivot(int64_t n, int64_t k, double* __restrict__ A,
                                                   int64_t lda, int64_t* __restrict__ piv, int64_t j0, int64_t j1) {
  __shared__ double sv[1024];
  __shared__ int64_t si[1024];
  const int tid = threadIdx.x;
  double best = -1.0;
  int64_t bi = k;
  for (int64_t i = k + tid; i < n; i += 1024) {
    double v = fabs(A[k * lda + i]);
    if (v > best) { best = v; bi = i; }
  }
  sv[tid] = best; si[tid] = bi;
  __syncthreads();
  for (int s = 512; s > 0; s >>= 1) {
    if (tid < s) {
      if (sv[tid + s] > sv[tid] || (sv[tid + s] == sv[tid] && si[tid + s] < si[tid])) {
        sv[tid] = sv[tid + s]; si[tid] = si[tid + s];
      }
    }
    __syncthreads();
  }
  const int64_t p = si[0];
  const double pv = sv[0];
  if (!(pv > 0.0)) {
    if (tid == 0) piv[k] = -1 - k;
    for (int64_t i = k + 1 + tid; i < n; i += 1024) A[k * lda + i] = 0.0;   // no L contribution
    return;
  }
  // swap rows k and p in columns [j0, j1) (the panel; k_laswp does the others)
  if (p != k) {
    for (int64_t j = j0 + tid; j < j1; j += 1024) {
      double t = A[j * lda + k];
      A[j * lda + k] = A[j * lda + p];
      A[j * lda + p] = t;
    }
  }
  if (tid == 0) piv[k] = p;
  __syncthreads();
  const double d = A[k * lda + k];
  for (int64_t i = k + 1 + tid; i < n; i += 1024) A[k * lda + i] /= d;
}

// rank-1 update of the panel columns (k, j1)
__global__ __launch_bounds__(256) void k_lu_update(int64_t n, int64_t k, double* __restrict__ A,
                                                   int64_t lda, const int64_t* __restrict__ piv, int64_t j1) {
  if (piv[k] < 0) return;
  const int64_t j = k + 1 + blockIdx.y;
  const int64_t i = k + 1 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= j1 || i >= n) return;
  const double ukj = A[j * lda + k];
  if (ukj != 0.0) A[j * lda + i] -= A[k * lda + i] * ukj;
}

// the panel's swaps (rows k0 .. k0+kb-1, in order) applied to columns outside [k0, k0+kb)
__global__ __launch_bounds__(256) void k_laswp(int64_t n, int64_t k0, int64_t kb, double* __restrict__ A,
                                               int64_t lda, const int64_t* __restrict__ piv) {
  int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n - kb) return;
  if (j >= k0) j += kb;
  double* col = A + j * lda;
  for (int64_t k = k0; k < k0 + kb; ++k) {
    const int64_t p = piv[k];
    if (p >= 0 && p != k) {
      const double t = col[k];
      col[k] = col[p];
      col[p] = t;
    }
  }
}

// U12 = L11^-1 A12 (unit lower L11 = rows/cols k0..k0+kb of A) for columns j >= k0 + kb, written in
// place and also to T (kb x m, k-major: T[q * ldt + jj]) -- the GEMM operand of the trailing update
__global__ __launch_bounds__(256) void k_lu_trsm(int64_t n, int64_t k0, int64_t kb, double* __restrict__ A,
                                                 int64_t lda, double* __restrict__ T, int64_t ldt) {
  __shared__ double sL[LU_NB * LU_NB];
  for (int64_t e = threadIdx.x; e < kb * kb; e += 256) {
    const int64_t c = e / kb, r = e - c * kb;
    sL[c * LU_NB + r] = A[(k0 + c) * lda + k0 + r];
  }
  __syncthreads();
  const int64_t jj = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t j = k0 + kb + jj;
  if (j >= n) return;
  double* col = A + j * lda + k0;
  double x[LU_NB];
#pragma unroll
  for (int q = 0; q < LU_NB; ++q) {
    if (q < kb) {
      double v = col[q];
      for (int r = 0; r < q; ++r) v = fma(-sL[r * LU_NB + q], x[r], v);
      x[q] = v;
      col[q] = v;
      T[q * ldt + jj] = v;
    }
  }
}

void getrf(hipStream_t st, int64_t n, double* A, int64_t lda, int64_t* piv, int* info, double* ws) {
  hipMemsetAsync(info, 0, sizeof(int), st);
  for (int64_t k0 = 0; k0 < n; k0 += LU_NB) {
    const int64_t kb = std::min<int64_t>(LU_NB, n - k0), j1 = k0 + kb;
    for (int64_t k = k0; k < j1; ++k) {
      hipLaunchKernelGGL(k_lu_pivot, dim3(1), dim3(1024), 0, st, n, k, A, lda, piv, k0, j1);
      if (k + 1 < j1 && k + 1 < n) {
        dim3 g((unsigned)cdiv(n - k - 1, 256), (unsigned)(j1 - k - 1));
        hipLaunchKernelGGL(k_lu_update, g, dim3(256), 0, st, n, k, A, lda, piv, j1);
      }
    }
    if (n - kb > 0) hipLaunchKernelGGL(k_laswp, dim3((unsigned)cdiv(n - kb, 256)), dim3(256), 0, st, n, k0, kb, A, lda, piv);
    const int64_t m = n - j1;
    if (m <= 0) continue;
    hipLaunchKernelGGL(k_lu_trsm, dim3((unsigned)cdiv(m, 256)), dim3(256), 0, st, n, k0, kb, A, lda, ws, m);
    // A22 -= L21 U12: C(i, j) -= sum_q X[q][i] Y[q][j], X = L21 (column q of A, k-major), Y = T
    GemmArgs g;
    g.ni = g.nj = m;
    g.K = kb;
    g.X = A + k0 * lda + j1;
    g.ldx = lda;
    g.Y = ws;
    g.ldy = m;
    g.C = A + j1 * lda + j1;
    g.ldc = lda;
    g.sub = 1;
    mfma_gemm_launch(st, g);
  }
}

// B row-major n x nrhs; single workgroup per rhs column (fallback path)
__global__ __launch_bounds__(256) void k_lu_solve(int64_t n, int64_t nrhs, const double* __restrict__ LU,
                                                  int64_t lda, const int64_t* __restrict__ piv,
                                                  double* __restrict__ B, int64_t ldb) {
  const int64_t c = blockIdx.x;
  const int tid = threadIdx.x;
  // apply row swaps
  if (tid == 0) {
    for (int64_t k = 0; k < n; ++k) {
      const int64_t p = piv[k];
      if (p >= 0 && p != k) {
        double t = B[k * ldb + c]; B[k * ldb + c] = B[p * ldb + c]; B[p * ldb + c] = t;
      }
    }
  }
  __syncthreads();
  // forward (unit lower)
  for (int64_t k = 0; k < n; ++k) {
    if (piv[k] < 0) continue;
    const double bk = B[k * ldb + c];
    for (int64_t i = k + 1 + tid; i < n; i += 256) B[i * ldb + c] -= LU[k * lda + i] * bk;
    __syncthreads();
  }
  // backward (upper)
  for (int64_t k = n - 1; k >= 0; --k) {
    __syncthreads();
    if (piv[k] < 0) {
      if (tid == 0) B[k * ldb + c] = 0.0;
      __syncthreads();
      continue;
    }
    if (tid == 0) B[k * ldb + c] /= LU[k * lda + k];
    __syncthreads();
    const double xk = B[k * ldb + c];
    for (int64_t i = tid; i < k; i += 256) B[i * ldb + c] -= LU[k * lda + i] * xk;
  }
}

void getrs(hipStream_t st, int64_t n, int64_t nrhs, const double* LU, int64_t lda, const int64_t* piv,
           double* B, int64_t ldb) {
  if (nrhs <= 0) return;
  hipLaunchKernelGGL(k_lu_solve, dim3(nrhs), dim3(256), 0, st, n, nrhs, LU, lda, piv, B, ldb);
}

// =====================================================================================
// small helpers
// =====================================================================================
__global__ void k_fill(double* p, int64_t n, double v) {
  int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) p[i] = v;
}
void fill(hipStream_t st, double* p, int64_t n, double v) {
  if (n > 0) hipLaunchKernelGGL(k_fill, dim3(cdiv(n, 256)), dim3(256), 0, st, p, n, v);
}
void copy(hipStream_t st, double* dst, const double* src, int64_t n) {
  if (n > 0) hipMemcpyAsync(dst, src, n * sizeof(double), hipMemcpyDeviceToDevice, st);
}

__global__ void k_sym_full(int64_t n, const double* L, int64_t ldl, double* out, int64_t ldo) {
  const int64_t j = blockIdx.y;                         // output row
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;  // output col
  if (i >= n) return;
  // out[j][i] = H(max(i,j), min(i,j)) ; lower col-major element (r, c) at c*ldl + r
  const int64_t r = i > j ? i : j, c = i > j ? j : i;
  out[j * ldo + i] = L[c * ldl + r];
}
void sym_lower_to_full(hipStream_t st, int64_t n, const double* L, int64_t ldl, double* out, int64_t ldo) {
  if (n <= 0) return;
  hipLaunchKernelGGL(k_sym_full, dim3(cdiv(n, 256), n), dim3(256), 0, st, n, L, ldl, out, ldo);
}

__global__ void k_transpose(int64_t rows, int64_t cols, const double* in, int64_t ldi, double* out,
                            int64_t ldo) {
  __shared__ double t[32][33];
  const int64_t bx = (int64_t)blockIdx.x * 32, by = (int64_t)blockIdx.y * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 256 threads: 32 x 8
  for (int k = ty; k < 32; k += 8) {
    const int64_t r = by + k, c = bx + tx;
    t[k][tx] = (r < rows && c < cols) ? in[r * ldi + c] : 0.0;
  }
  __syncthreads();
  for (int k = ty; k < 32; k += 8) {
    const int64_t r = bx + k, c = by + tx;  // out row = in col
    if (r < cols && c < rows) out[r * ldo + c] = t[tx][k];
  }
}
void transpose(hipStream_t st, int64_t rows, int64_t cols, const double* in, int64_t ldi, double* out,
               int64_t ldo) {
  if (rows <= 0 || cols <= 0) return;
  hipLaunchKernelGGL(k_transpose, dim3(cdiv(cols, 32), cdiv(rows, 32)), dim3(256), 0, st, rows, cols,
                     in, ldi, out, ldo);
}

}  // namespace ipm
