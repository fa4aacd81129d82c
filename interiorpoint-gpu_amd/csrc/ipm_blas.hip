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
#include "ipm_common.h"

#include <algorithm>
#include <cmath>

namespace ipm {

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

// =====================================================================================
// GEMV (row-major M):  y = alpha * M x + beta * y        one wave per row
// =====================================================================================
template <bool VEC>
__global__ __launch_bounds__(256) void k_gemv_n(int64_t rows, int64_t cols, double alpha,
                                                const double* __restrict__ M, int64_t ldm,
                                                const double* __restrict__ x, double beta,
                                                double* __restrict__ y) {
  const int lane = threadIdx.x & 63;
  const int64_t row = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const double* mr = M + row * ldm;
  double acc0 = 0.0, acc1 = 0.0;
  if (VEC) {
    const int64_t c2 = cols >> 1;
    const double2* m2 = reinterpret_cast<const double2*>(mr);
    const double2* x2 = reinterpret_cast<const double2*>(x);
    for (int64_t j = lane; j < c2; j += 64) {
      double2 a = m2[j], b = x2[j];
      acc0 = fma(a.x, b.x, acc0);
      acc1 = fma(a.y, b.y, acc1);
    }
    if ((cols & 1) && lane == 0) acc0 = fma(mr[cols - 1], x[cols - 1], acc0);
  } else {
    for (int64_t j = lane; j < cols; j += 64) acc0 = fma(mr[j], x[j], acc0);
  }
  double s = wave_sum(acc0 + acc1);
  if (lane == 0) y[row] = (beta == 0.0) ? alpha * s : alpha * s + beta * y[row];
}

void gemv_n(hipStream_t st, int64_t rows, int64_t cols, double alpha, const double* M, int64_t ldm,
            const double* x, double beta, double* y) {
  if (rows <= 0) return;
  dim3 g(cdiv(rows, 4)), b(256);
  bool vec = ((ldm & 1) == 0) && ((((uintptr_t)M) & 15) == 0) && ((((uintptr_t)x) & 15) == 0);
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
  for (int64_t c = 0; c < nchunk; ++c) s += part[c * cols + j];
  y[j] = (beta == 0.0) ? alpha * s : alpha * s + beta * y[j];
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

// =====================================================================================
// SYRK / GEMM^T on fp64 MFMA (v_mfma_f64_16x16x4_f64)
//
//   H(i,j) = alpha * sum_k w[k] X[k][i] Y[k][j] + beta*H(i,j) + tP*P[j][i] + [i==j] dvec[i]
//   for the lower triangle i >= j; H column-major (element (i,j) at j*ldh + i).
//
// 128x128 output tile per 256-thread workgroup (2x2 waves of 64x64 = 4x4 MFMA tiles),
// K staged 16 rows at a time through LDS (register prefetch of the next K-slab).
// f64 MFMA fragment maps (cdna_hip_programming.md §3): A: lane l holds A[l&15][l>>4];
// B: lane l holds B[l>>4][l&15]; D: lane l holds D[(l>>4)+4r][l&15], r=0..3.
// We put j (the output column) on the MFMA row and i (output row) on the MFMA column so that
// 16 consecutive lanes store 16 consecutive doubles of a column-major H column.
// =====================================================================================
constexpr int SK_BN = 128;   // output tile
constexpr int SK_BK = 16;    // K slab
constexpr int SK_LDS = 144;  // padded LDS row (doubles): 288 dwords == 32 mod 64 -> no 2-way conflict

template <bool VEC, bool SYM>
__global__ __launch_bounds__(256, 1) void k_syrk_lower(
    int64_t n, int64_t K, double alpha, const double* __restrict__ X, int64_t ldx,
    const double* __restrict__ Y, int64_t ldy, const double* __restrict__ w, double beta,
    double* __restrict__ H, int64_t ldh, const double* __restrict__ P, int64_t ldp, double tP,
    const double* __restrict__ dvec, const int* __restrict__ info, int64_t tiles_n) {
  if (info && *info != 0) return;
  // lower-triangular tile index -> (bi >= bj)
  const int64_t L = blockIdx.x;
  int64_t bi = (int64_t)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
  while ((bi + 1) * (bi + 2) / 2 <= L) ++bi;
  while (bi * (bi + 1) / 2 > L) --bi;
  const int64_t bj = L - bi * (bi + 1) / 2;
  const int64_t I0 = bi * SK_BN, J0 = bj * SK_BN;

  __shared__ double sX[2][SK_BK * SK_LDS];  // i side (weighted)
  __shared__ double sY[2][SK_BK * SK_LDS];  // j side

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wj = wv >> 1, wi = wv & 1;
  // staging assignment: row r = tid>>4 (0..15), 8 consecutive columns from (tid&15)*8
  const int sr = tid >> 4, sc = (tid & 15) * 8;

  dbl4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};

  double rx[8], ry[8];
  auto load_slab = [&](int64_t k0) {
    const int64_t k = k0 + sr;
    const bool kin = k < K;
    const double wk = (kin && w) ? w[k] : 1.0;
    const double* xr = X + k * ldx;
    const double* yr = (SYM ? X : Y) + k * (SYM ? ldx : ldy);
    if (VEC && kin && I0 + sc + 8 <= n && J0 + sc + 8 <= n) {
      const double2* x2 = reinterpret_cast<const double2*>(xr + I0 + sc);
      const double2* y2 = reinterpret_cast<const double2*>(yr + J0 + sc);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double2 a = x2[q], b = y2[q];
        rx[2 * q] = a.x * wk; rx[2 * q + 1] = a.y * wk;
        ry[2 * q] = b.x; ry[2 * q + 1] = b.y;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        const int64_t ci = I0 + sc + q, cj = J0 + sc + q;
        rx[q] = (kin && ci < n) ? xr[ci] * wk : 0.0;
        ry[q] = (kin && cj < n) ? yr[cj] : 0.0;
      }
    }
  };
  auto store_slab = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sX[buf][sr * SK_LDS + sc + q] = rx[q];
      sY[buf][sr * SK_LDS + sc + q] = ry[q];
    }
  };

  const int64_t nslab = (K + SK_BK - 1) / SK_BK;
  if (nslab > 0) {
    load_slab(0);
    store_slab(0);
  }
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int64_t s = 0; s < nslab; ++s) {
    const int buf = s & 1;
    if (s + 1 < nslab) load_slab((s + 1) * SK_BK);
#pragma unroll
    for (int kk = 0; kk < SK_BK / 4; ++kk) {
      const int krow = (kk * 4 + fk) * SK_LDS;
      double a[4], b[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = sY[buf][krow + wj * 64 + t * 16 + fr];
        b[t] = sX[buf][krow + wi * 64 + t * 16 + fr];
      }
#pragma unroll
      for (int tj = 0; tj < 4; ++tj)
#pragma unroll
        for (int ti = 0; ti < 4; ++ti)
          acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[tj], b[ti], acc[tj][ti], 0, 0, 0);
    }
    if (s + 1 < nslab) store_slab(buf ^ 1);
    __syncthreads();
  }

  // epilogue: lower triangle only
#pragma unroll
  for (int tj = 0; tj < 4; ++tj) {
#pragma unroll
    for (int ti = 0; ti < 4; ++ti) {
      const int64_t i = I0 + wi * 64 + ti * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t j = J0 + wj * 64 + tj * 16 + fk + 4 * r;
        if (i < n && j < n && i >= j) {
          double v = alpha * acc[tj][ti][r];
          double* hp = H + j * ldh + i;
          if (beta != 0.0) v += beta * (*hp);
          if (P) v += tP * P[j * ldp + i];
          if (dvec && i == j) v += dvec[i];
          *hp = v;
        }
      }
    }
  }
}

static void syrk_launch(hipStream_t st, int64_t n, int64_t k, double alpha, const double* X,
                        int64_t ldx, const double* Y, int64_t ldy, const double* w, double beta,
                        double* H, int64_t ldh, const SyrkEpi& e, const int* info) {
  if (n <= 0) return;
  const int64_t T = cdiv(n, SK_BN);
  const int64_t nblk = T * (T + 1) / 2;
  const bool sym = (Y == nullptr) || (Y == X && ldy == ldx);
  bool vec = ((ldx & 1) == 0) && ((((uintptr_t)X) & 15) == 0);
  if (!sym) vec = vec && ((ldy & 1) == 0) && ((((uintptr_t)Y) & 15) == 0);
  dim3 g(nblk), b(256);
#define SK_ARGS n, k, alpha, X, ldx, Y, ldy, w, beta, H, ldh, e.P, e.ldp, e.tP, e.dvec, info, T
  if (sym) {
    if (vec) hipLaunchKernelGGL((k_syrk_lower<true, true>), g, b, 0, st, SK_ARGS);
    else hipLaunchKernelGGL((k_syrk_lower<false, true>), g, b, 0, st, SK_ARGS);
  } else {
    if (vec) hipLaunchKernelGGL((k_syrk_lower<true, false>), g, b, 0, st, SK_ARGS);
    else hipLaunchKernelGGL((k_syrk_lower<false, false>), g, b, 0, st, SK_ARGS);
  }
#undef SK_ARGS
}

void syrk_lower(hipStream_t st, int64_t n, int64_t k, double alpha, const double* X, int64_t ldx,
                const double* Y, int64_t ldy, const double* w, double beta, double* H, int64_t ldh,
                const SyrkEpi& epi) {
  syrk_launch(st, n, k, alpha, X, ldx, Y, ldy, w, beta, H, ldh, epi, nullptr);
}

// =====================================================================================
// General GEMM update on MFMA:  C(m x n, col-major) -= A(m x k, col-major) B(n x k, col-major)^T
// (Cholesky sub-panel update).  Same 128x128 tile / 16-deep slab scheme as the SYRK.
// Operands viewed as "k-major rows": A^T row p = column p of A (contiguous in m).
// =====================================================================================
template <bool VEC>
__global__ __launch_bounds__(256, 1) void k_gemm_nt_sub(int64_t m, int64_t n, int64_t K,
                                                        const double* __restrict__ A, int64_t lda,
                                                        const double* __restrict__ B, int64_t ldb,
                                                        double* __restrict__ C, int64_t ldc,
                                                        const int* __restrict__ info,
                                                        int64_t tiles_m) {
  if (info && *info != 0) return;
  const int64_t bi = blockIdx.x % tiles_m, bj = blockIdx.x / tiles_m;
  const int64_t I0 = bi * SK_BN, J0 = bj * SK_BN;
  __shared__ double sA[2][SK_BK * SK_LDS];
  __shared__ double sB[2][SK_BK * SK_LDS];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wj = wv >> 1, wi = wv & 1;
  const int sr = tid >> 4, sc = (tid & 15) * 8;
  dbl4 acc[4][4];
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = dbl4{0.0, 0.0, 0.0, 0.0};
  double ra[8], rb[8];
  auto load_slab = [&](int64_t k0) {
    const int64_t k = k0 + sr;
    const bool kin = k < K;
    const double* ar = A + k * lda;
    const double* br = B + k * ldb;
    if (VEC && kin && I0 + sc + 8 <= m && J0 + sc + 8 <= n) {
      const double2* a2 = reinterpret_cast<const double2*>(ar + I0 + sc);
      const double2* b2 = reinterpret_cast<const double2*>(br + J0 + sc);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        double2 a = a2[q], b = b2[q];
        ra[2 * q] = a.x; ra[2 * q + 1] = a.y;
        rb[2 * q] = b.x; rb[2 * q + 1] = b.y;
      }
    } else {
#pragma unroll
      for (int q = 0; q < 8; ++q) {
        ra[q] = (kin && I0 + sc + q < m) ? ar[I0 + sc + q] : 0.0;
        rb[q] = (kin && J0 + sc + q < n) ? br[J0 + sc + q] : 0.0;
      }
    }
  };
  auto store_slab = [&](int buf) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      sA[buf][sr * SK_LDS + sc + q] = ra[q];
      sB[buf][sr * SK_LDS + sc + q] = rb[q];
    }
  };
  const int64_t nslab = (K + SK_BK - 1) / SK_BK;
  if (nslab > 0) { load_slab(0); store_slab(0); }
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int64_t s = 0; s < nslab; ++s) {
    const int buf = s & 1;
    if (s + 1 < nslab) load_slab((s + 1) * SK_BK);
#pragma unroll
    for (int kk = 0; kk < SK_BK / 4; ++kk) {
      const int krow = (kk * 4 + fk) * SK_LDS;
      double a[4], b[4];
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        a[t] = sB[buf][krow + wj * 64 + t * 16 + fr];
        b[t] = sA[buf][krow + wi * 64 + t * 16 + fr];
      }
#pragma unroll
      for (int tj = 0; tj < 4; ++tj)
#pragma unroll
        for (int ti = 0; ti < 4; ++ti)
          acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[tj], b[ti], acc[tj][ti], 0, 0, 0);
    }
    if (s + 1 < nslab) store_slab(buf ^ 1);
    __syncthreads();
  }
#pragma unroll
  for (int tj = 0; tj < 4; ++tj)
#pragma unroll
    for (int ti = 0; ti < 4; ++ti) {
      const int64_t i = I0 + wi * 64 + ti * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t j = J0 + wj * 64 + tj * 16 + fk + 4 * r;
        if (i < m && j < n) C[j * ldc + i] -= acc[tj][ti][r];
      }
    }
}

static void gemm_nt_sub_launch(hipStream_t st, int64_t m, int64_t n, int64_t k, const double* A,
                               int64_t lda, const double* B, int64_t ldb, double* C, int64_t ldc,
                               const int* info) {
  if (m <= 0 || n <= 0 || k <= 0) return;
  const int64_t tm = cdiv(m, SK_BN), tn = cdiv(n, SK_BN);
  bool vec = ((lda & 1) == 0) && ((ldb & 1) == 0) && ((((uintptr_t)A) & 15) == 0) &&
             ((((uintptr_t)B) & 15) == 0);
  dim3 g(tm * tn), b(256);
  if (vec)
    hipLaunchKernelGGL(k_gemm_nt_sub<true>, g, b, 0, st, m, n, k, A, lda, B, ldb, C, ldc, info, tm);
  else
    hipLaunchKernelGGL(k_gemm_nt_sub<false>, g, b, 0, st, m, n, k, A, lda, B, ldb, C, ldc, info, tm);
}

void gemm_nt_sub(hipStream_t st, int64_t m, int64_t n, int64_t k, const double* A, int64_t lda,
                 const double* B, int64_t ldb, double* C, int64_t ldc) {
  gemm_nt_sub_launch(st, m, n, k, A, lda, B, ldb, C, ldc, nullptr);
}

// =====================================================================================
// Cholesky panel: factor the nb x nb diagonal block and solve the rows below it.
// Every workgroup factors the diagonal block redundantly in LDS (no inter-workgroup
// hand-off); workgroup 0 writes L11 back, workgroups g >= 1 each solve 64 rows of
// L21 = A21 L11^{-T}.  LAPACK potrf failure rule: pivot <= 0 or NaN -> info = column.
// =====================================================================================
constexpr int PF_NB = 64;    // panel width
constexpr int PF_RB = 64;    // rows per workgroup for the TRSM part
constexpr int PF_LD = PF_NB + 1;

__global__ __launch_bounds__(256) void k_potrf_panel(int64_t n, int64_t k0, int nb, double* __restrict__ A,
                                                     int64_t lda, int* __restrict__ info) {
  if (*info != 0) return;
  __shared__ double sL[PF_NB * PF_LD];
  __shared__ double sR[PF_RB * PF_LD];
  __shared__ int fail;
  const int tid = threadIdx.x;
  if (tid == 0) fail = 0;
  // load the diagonal block (lower part) column-major -> sL[i*LD + j] (row i, col j)
  for (int idx = tid; idx < nb * nb; idx += 256) {
    const int j = idx / nb, i = idx % nb;
    sL[i * PF_LD + j] = (i >= j) ? A[(k0 + j) * lda + k0 + i] : 0.0;
  }
  __syncthreads();
  // right-looking factorisation: thread t owns row i = t (t < nb)
  for (int j = 0; j < nb; ++j) {
    double djj = sL[j * PF_LD + j];
    if (!(djj > 0.0)) {  // <= 0 or NaN
      if (tid == 0) fail = j + 1;
      break;
    }
    djj = sqrt(djj);
    __syncthreads();
    if (tid == j) sL[j * PF_LD + j] = djj;
    if (tid > j && tid < nb) sL[tid * PF_LD + j] /= djj;
    __syncthreads();
    if (tid > j && tid < nb) {
      const double lij = sL[tid * PF_LD + j];
      for (int l = j + 1; l <= tid; ++l) sL[tid * PF_LD + l] -= lij * sL[l * PF_LD + j];
    }
    __syncthreads();
  }
  __syncthreads();
  if (fail) {
    if (blockIdx.x == 0 && tid == 0) atomicCAS(info, 0, (int)(k0 + fail));
    return;
  }
  if (blockIdx.x == 0) {
    for (int idx = tid; idx < nb * nb; idx += 256) {
      const int j = idx / nb, i = idx % nb;
      if (i >= j) A[(k0 + j) * lda + k0 + i] = sL[i * PF_LD + j];
    }
    return;
  }
  // rows below: r0 = k0 + nb + (g-1)*RB
  const int64_t r0 = k0 + nb + (int64_t)(blockIdx.x - 1) * PF_RB;
  const int rows = (int)min((int64_t)PF_RB, n - r0);
  if (rows <= 0) return;
  for (int idx = tid; idx < rows * nb; idx += 256) {
    const int j = idx / rows, r = idx % rows;
    sR[r * PF_LD + j] = A[(k0 + j) * lda + r0 + r];
  }
  __syncthreads();
  // solve X L11^T = R : thread layout r = tid & 63, column group q = tid >> 6
  const int r = tid & 63, q = tid >> 6;
  for (int j = 0; j < nb; ++j) {
    if (r < rows && q == (j & 3)) sR[r * PF_LD + j] /= sL[j * PF_LD + j];
    __syncthreads();
    if (r < rows) {
      const double xj = sR[r * PF_LD + j];
      for (int l = j + 1 + ((q - (j + 1)) & 3); l < nb; l += 4) sR[r * PF_LD + l] -= xj * sL[l * PF_LD + j];
    }
    __syncthreads();
  }
  for (int idx = tid; idx < rows * nb; idx += 256) {
    const int j = idx / rows, rr = idx % rows;
    A[(k0 + j) * lda + r0 + rr] = sR[rr * PF_LD + j];
  }
}

void potrf_lower(hipStream_t st, int64_t n, double* A, int64_t lda, int* info) {
  hipMemsetAsync(info, 0, sizeof(int), st);
  for (int64_t k = 0; k < n; k += PF_NB) {
    const int nb = (int)std::min<int64_t>(PF_NB, n - k);
    const int64_t below = n - k - nb;
    dim3 g(1 + cdiv(std::max<int64_t>(below, 0), PF_RB));
    hipLaunchKernelGGL(k_potrf_panel, g, dim3(256), 0, st, n, k, nb, A, lda, info);
    if (below > 0) {
      // trailing update A22 -= L21 L21^T : X = L21^T viewed as k-major rows (col p of L21)
      SyrkEpi e;
      syrk_launch(st, below, nb, -1.0, A + k * lda + (k + nb), lda, nullptr, 0, nullptr, 1.0,
                  A + (k + nb) * lda + (k + nb), lda, e, info);
    }
  }
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

// L L^T X = B in place; W: scratch n x nrhs (ldb)
void potrs_lower(hipStream_t st, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B,
                 int64_t ldb, double* W) {
  trsm_lower_fwd(st, n, nrhs, L, ldl, B, ldb, W);
  trsm_lower_bwd(st, n, nrhs, L, ldl, W, ldb, B);
}

// =====================================================================================
// LU with partial pivoting (column-major A, in place), right-looking, one column per step.
// Fallback path only (after a Cholesky failure).  A zero pivot column is recorded with
// piv = -1 - row and skipped; getrs then sets that unknown to 0 (the minimum-norm choice
// when the null space is that coordinate -- see DESIGN.md, fallback semantics).
// =====================================================================================
__global__ __launch_bounds__(1024) void k_lu_pivot(int64_t n, int64_t k, double* __restrict__ A,
                                                   int64_t lda, int64_t* __restrict__ piv) {
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
    return;
  }
  // swap rows k and p across all columns
  if (p != k) {
    for (int64_t j = tid; j < n; j += 1024) {
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

__global__ __launch_bounds__(256) void k_lu_update(int64_t n, int64_t k, double* __restrict__ A,
                                                   int64_t lda, const int64_t* __restrict__ piv) {
  if (piv[k] < 0) return;
  const int64_t j = k + 1 + blockIdx.y;
  const int64_t i = k + 1 + (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n || i >= n) return;
  const double ukj = A[j * lda + k];
  if (ukj != 0.0) A[j * lda + i] -= A[k * lda + i] * ukj;
}

void getrf(hipStream_t st, int64_t n, double* A, int64_t lda, int64_t* piv, int* info) {
  hipMemsetAsync(info, 0, sizeof(int), st);
  for (int64_t k = 0; k < n; ++k) {
    hipLaunchKernelGGL(k_lu_pivot, dim3(1), dim3(1024), 0, st, n, k, A, lda, piv);
    if (k + 1 < n) {
      dim3 g(cdiv(n - k - 1, 256), n - k - 1);
      hipLaunchKernelGGL(k_lu_update, g, dim3(256), 0, st, n, k, A, lda, piv);
    }
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
