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
#include "ipm_mfma.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>

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
// SYRK / GEMM^T on fp64 MFMA: the tile kernel lives in ipm_mfma.h (k_mfma_gemm).
//   H(i,j) = alpha * sum_k w[k] X[k][i] Y[k][j] + beta*H(i,j) + tP*P[j][i] + [i==j] dvec[i]
//   for the lower triangle i >= j; H column-major (element (i,j) at j*ldh + i).
// =====================================================================================
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
  mfma_gemm_launch(st, a);
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

__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(
      reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
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

#ifdef IPM_STAMPS
__device__ unsigned long long ipm_stamps[64];
#define STAMP() do { if (tid == 0) ipm_stamps[nst] = __builtin_amdgcn_s_memtime(); ++nst; } while (0)
#else
#define STAMP() do {} while (0)
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
  }
  if (lane < 16) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      if (sc1) st_sc1(&out[c * 16 + r], x[r]);
      else out[c * 16 + r] = x[r];
    }
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
  double sLr[256];       // L_JJ row-major (broadcast reads of its rows)
  double srinv[8 * 16];  // 1 / L_cc per diagonal block
  double scol[2][16];    // leaf column broadcast
  int fail;
};

__device__ __forceinline__ void diag_role(int64_t k0, int nb, double* __restrict__ A, int64_t lda,
                                          double* __restrict__ dinv_out, int* __restrict__ info,
                                          double* pubL, unsigned* progress, DiagSmem& sm) {
  double* sD = sm.sD;
  double* sLr = sm.sLr;
  double* srinv = sm.srinv;
  auto& scol = sm.scol;
  int& fail = sm.fail;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;   // 4 waves
  const int fr = lane & 15, fk = lane >> 4;
#ifdef IPM_STAMPS
  int nst = 0;
#endif
  if (tid == 0) fail = 0;
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
                                             16, 0, 0);
          }
    if (*info != 0) return;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else {
    // ---- partial panel (last one): register path with identity padding beyond nb
    const bool vec = ((lda & 1) == 0) && ((k0 & 1) == 0);
    const int ic0 = min(i0, nb - 1), ic1 = min(i0 + 1, nb - 1);
    const double* base = A + k0 * lda + k0;
    double2 v[32];
    if (vec && i0 + 1 < nb) {
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const int jc = min(jb + 4 * q, nb - 1);
        v[q] = *reinterpret_cast<const double2*>(base + jc * lda + i0);
      }
    } else {
#pragma unroll
      for (int q = 0; q < 32; ++q) {
        const int jc = min(jb + 4 * q, nb - 1);
        v[q].x = base[jc * lda + ic0];
        v[q].y = base[jc * lda + ic1];
      }
    }
    if (*info != 0) return;
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
  for (int J = 0; J < 8; ++J) {
    // ---- 1. left-looking update of block column J: T_IJ -= sum_{P<J} L_IP L_JP^T, I >= J
    //      wave 0 updates the diagonal tile and goes straight on to factor it; waves 1-3 update
    //      the tiles below meanwhile (no barrier in between)
    for (int tI = (wv == 0 ? 0 : wv); J > 0 && tI < 8 - J; tI += (wv == 0 ? 8 : 3)) {
      const int I = J + tI;
      const int cb = bidx(I, J) * 256 + fk * 16 + fr;
      dbl4 acc[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int r = 0; r < 4; ++r) acc[0][r] = sD[cb + 64 * r];
      for (int P = 0; P < J; ++P) {
        const int ab = bidx(J, P) * 256 + fk * 16 + fr, bb = bidx(I, P) * 256 + fk * 16 + fr;
        double av[4], bv[4];
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) {
          av[s4] = -sD[ab + 64 * s4];
          bv[s4] = sD[bb + 64 * s4];
        }
#pragma unroll
        for (int s4 = 0; s4 < 4; ++s4) acc[s4] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[s4], bv[s4], acc[s4], 0, 0, 0);
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) sD[cb + 64 * r] = (acc[0][r] + acc[1][r]) + (acc[2][r] + acc[3][r]);
    }
    STAMP();
    // ---- 2. wave 0: factor the 16 x 16 block (J,J) in registers, lane r = row r.
    //      Right-looking with NO lane masks: entries above the diagonal (lane r < column c)
    //      turn into garbage but are never read -- every broadcast reads lane c2 > c or the
    //      pivot lane.  sqrt and reciprocal come from one rsqrt (off one chain).
    if (wv == 0) {
      const int db = bidx(J, J) * 256;
      const int rr = lane & 15;
      double row[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) row[c] = sD[db + c * 16 + rr];
      // Column c+1 is updated first (readlane broadcast) and ITS pivot's rsqrt issued; the rest of
      // column c's rank-1 update reads column c from an LDS copy (one write, four 32-byte reads
      // instead of 2 readlanes per element) and fills the rsqrt latency.
      // Column c+1 is updated first (readlane broadcast) and ITS pivot's rsqrt issued; the rest of
      // column c's rank-1 update reads column c from an LDS copy (one write, a few wide reads
      // instead of 2 readlanes per element) and fills the rsqrt latency.
      int bad = 0;
      double piv = readlane_d(row[0], 0);
      double dv = rsqrt_pivot(piv);
      double dvs[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (!(piv > 0.0) && bad == 0) bad = c + 1;
        dvs[c] = dv;
        row[c] *= dv;                      // lane c: piv * dv = L_cc
        scol[c & 1][rr] = row[c];          // lanes 16-63 duplicate rows: same value, same address
        double pivn = 1.0, dvn = 1.0;
        if (c + 1 < 16) {
          row[c + 1] = fma(-row[c], readlane_d(row[c], c + 1), row[c + 1]);
          pivn = readlane_d(row[c + 1], c + 1);
          dvn = rsqrt_pivot(pivn);
        }
        // (same-wave LDS write -> read: in order, no barrier needed; the compiler keeps the order
        //  because the addresses may alias)
#pragma unroll
        for (int c2 = c + 2; c2 < 16; ++c2) row[c2] = fma(-row[c], scol[c & 1][c2], row[c2]);
        piv = pivn;
        dv = dvn;
      }
      if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 16; ++c)
          if (lane == c) srinv[J * 16 + c] = dvs[c];
      }
      if (lane < 16) {
#pragma unroll
        for (int c = 0; c < 16; ++c) {
          const double v = (rr >= c) ? row[c] : 0.0;
          sD[db + c * 16 + rr] = v;          // column-major block
          sLr[rr * 16 + c] = v;              // row-major copy
        }
      }
      if (lane == 0 && bad) fail = J * 16 + bad;
    } else if (wv == 3 && J > 0) {
      // meanwhile (off the chain) wave 3 inverts the PREVIOUS diagonal block for the row part
      tri_inverse16(&sD[bidx(J - 1, J - 1) * 256], &srinv[(J - 1) * 16], dinv_out + (J - 1) * 256, lane,
                    pubL != nullptr);
    } else if (wv == 2 && J > 0 && pubL) {
      // ... and wave 2 publishes the previous diagonal block (the chain wave stores nothing)
      const int db = bidx(J - 1, J - 1) * 256;
#pragma unroll
      for (int q = 0; q < 4; ++q) st_sc1(&pubL[db + q * 64 + lane], sD[db + q * 64 + lane]);
    }
    if (pubL) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    STAMP();
    if (fail) break;
    // block row J-1 of L11 and Dinv_{J-1} are stored: release them to the row workgroups
    if (pubL && tid == 0 && J > 0) __hip_atomic_store(progress, (unsigned)J, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    // ---- 3. tiles below: X = T L_JJ^-T by substitution, one thread per tile row:
    //      X[r][c] = (T[r][c] - sum_{k<c} X[r][k] L[c][k]) / L_cc
    if (tid < (7 - J) * 16) {
      const int I = J + 1 + (tid >> 4), r = tid & 15;
      const int cb = bidx(I, J) * 256 + r;
      double x[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) x[c] = sD[cb + c * 16];
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        double v = x[c];
#pragma unroll
        for (int k = 0; k < c; ++k) v = fma(-x[k], sLr[c * 16 + k], v);
        x[c] = v * srinv[J * 16 + c];
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) sD[cb + c * 16] = x[c];
      if (pubL) {
#pragma unroll
        for (int c = 0; c < 16; ++c) st_sc1(&pubL[cb + c * 16], x[c]);
      }
    }
    __syncthreads();
    STAMP();
  }
  if (fail) {
    if (tid == 0) {
      atomicCAS(info, 0, (int)(k0 + fail));
      // release the row workgroups (they finish on garbage; the failed factor is discarded)
      if (pubL) {
        __threadfence();
        __hip_atomic_store(progress, 0xFFFFFFFFu, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
    return;
  }
  if (wv == 3) tri_inverse16(&sD[bidx(7, 7) * 256], &srinv[7 * 16], dinv_out + 7 * 256, lane, pubL != nullptr);
  if (wv == 2 && pubL) {
    const int db = bidx(7, 7) * 256;
#pragma unroll
    for (int q = 0; q < 4; ++q) st_sc1(&pubL[db + q * 64 + lane], sD[db + q * 64 + lane]);
  }
  if (pubL) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(progress, 8u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // ---- write back L11 (lower part, i < nb, j < nb)
  {
    double* col = A + k0 * lda + k0 + i0;
#pragma unroll
    for (int q = 0; q < 32; ++q) {
      const int j = jb + 4 * q;
      if ((i0 >> 4) >= (j >> 4) && j < nb) {
        const double2 v = *reinterpret_cast<const double2*>(&sD[bidx(i0 >> 4, j >> 4) * 256 + (j & 15) * 16 + (i0 & 15)]);
        if (i0 >= j && i0 < nb) col[j * lda] = v.x;
        if (i0 + 1 >= j && i0 + 1 < nb) col[j * lda + 1] = v.y;
      }
    }
  }
  STAMP();
}
#undef STAMP

// Row role: rows below the diagonal block, L21 = A21 L11^-T, 64 rows per workgroup, 16 rows per
// wave.  Each wave runs the 8-step block forward substitution in MFMA registers,
//   X_J = (B_J - sum_{P<J} X_P L_JP^T) Dinv_J^T,
// starting step J as soon as the diagonal role has released block row J (*progress > J).
// L blocks and Dinv come from the producer's sc1 stores and are read with sc1 loads only.
__device__ __forceinline__ void row_role(int64_t chunk, int64_t n, int64_t k0, int nb, double* __restrict__ A,
                                         int64_t lda, const double* dinv, const double* pubL,
                                         unsigned* progress) {
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
      b[J][r] = (rin && c < nb) ? A[(k0 + c) * lda + row] : 0.0;
    }
  dbl4 x[8];
  unsigned known = 0;
#pragma unroll
  for (int J = 0; J < 8; ++J) {
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
  if (rin) {
#pragma unroll
    for (int J = 0; J < 8; ++J)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int c = J * 16 + fk + 4 * r;
        if (c < nb) A[(k0 + c) * lda + row] = x[J][r];
      }
  }
}

// One panel (width nb <= 128 at column k0) in ONE launch.  Workgroups draw tickets: ticket 0 is the
// diagonal role (so it is resident before anyone waits on it -- no deadlock for any residency),
// tickets 1.. are the row chunks, pipelined one block column behind the diagonal role.
// ctl: 2 zeroed words {ticket, progress}.
__global__ __launch_bounds__(256) void k_potrf_panel(int64_t n, int64_t k0, int nb, double* __restrict__ A,
                                                     int64_t lda, double* ws, unsigned* ctl, int* __restrict__ info) {
  __shared__ DiagSmem sm;
  __shared__ int sticket;
  if (threadIdx.x == 0) sticket = (int)atomicAdd(&ctl[0], 1u);
  __syncthreads();
  const int t = sticket;
  double* dinv = ws;
  double* pubL = ws + PF_DINV;
  if (t == 0) {
    diag_role(k0, nb, A, lda, dinv, info, pubL, &ctl[1], sm);
  } else {
    if (*info != 0) return;
    row_role(t - 1, n, k0, nb, A, lda, dinv, pubL, &ctl[1]);
  }
}

// one panel of width nb <= 128 at column k0 (ctl: this panel's 2 zeroed control words)
static void panel_launch(hipStream_t st, int64_t n, int64_t k0, int nb, double* A, int64_t lda, int* info,
                         double* ws, unsigned* ctl) {
  const int64_t below = n - k0 - nb;
  hipLaunchKernelGGL(k_potrf_panel, dim3(1 + cdiv(std::max<int64_t>(below, 0), PF_RB)), dim3(256), 0, st, n, k0,
                     nb, A, lda, ws, ctl, info);
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
// CUs kept free of trailing-update workgroups while a panel runs (IPM_PANEL_CUS, default 32; 0: off)
static int panel_reserve_cus() {
  static int r = -1;
  if (r < 0) {
    const char* e = getenv("IPM_PANEL_CUS");
    r = e ? atoi(e) : 32;
    if (r < 0 || r >= num_cus()) r = 0;
  }
  return r;
}

// Blocked right-looking Cholesky with one block of look-ahead.
//   side stream: factor block k (two 128-wide panels + the GEMM between them)
//   main stream: update block k+1's columns first, release it to the side stream, then the
//                rest of the trailing matrix (SYRK, K = 256) -- overlapped with block k+1's panel.
// Without a side stream (side == main) the same sequence runs in order.
void potrf_lower_la(hipStream_t caller, const PotrfStreams* pst, int64_t n, double* A, int64_t lda, int* info,
                    double* ws) {
  hipMemsetAsync(info, 0, sizeof(int), caller);
  unsigned* ctl = reinterpret_cast<unsigned*>(ws + PF_DINV + 36 * 256);   // 2 words per panel
  hipMemsetAsync(ctl, 0, 2 * sizeof(unsigned) * cdiv(std::max<int64_t>(n, 1), PF_NB), caller);
  const bool two = pst && pst->side;
  hipStream_t st = (two && pst->main) ? pst->main : caller;
  hipStream_t side = two ? pst->side : caller;
  hipEvent_t ev_rel = two ? pst->ev_rel : nullptr, ev_pan = two ? pst->ev_pan : nullptr;
  if (st != caller) { hipEventRecord(pst->ev_in, caller); hipStreamWaitEvent(st, pst->ev_in, 0); }
  if (two) { hipEventRecord(ev_rel, st); hipStreamWaitEvent(side, ev_rel, 0); }
  hipStream_t ps = two ? side : st;
  for (int64_t k0 = 0; k0 < n; k0 += CH_NB) {
    const int w = (int)std::min<int64_t>(CH_NB, n - k0);
    // ---- panel k on the side stream
    const int w1 = std::min(w, PF_NB);
    panel_launch(ps, n, k0, w1, A, lda, info, ws, ctl + 2 * (k0 / PF_NB));
    if (w > w1) {
      // A[k0+w1 : n, k0+w1 : k0+w] -= L[k0+w1 : n, k0 : k0+w1] L[k0+w1 : k0+w, k0 : k0+w1]^T
      gemm_nt_sub_launch(ps, n - k0 - w1, w - w1, w1, A + k0 * lda + k0 + w1, lda, A + k0 * lda + k0 + w1, lda,
                         A + (k0 + w1) * lda + k0 + w1, lda, info);
      panel_launch(ps, n, k0 + w1, w - w1, A, lda, info, ws, ctl + 2 * ((k0 + w1) / PF_NB));
    }
    if (two) { hipEventRecord(ev_pan, side); hipStreamWaitEvent(st, ev_pan, 0); }
    // ---- trailing update on the main stream
    const int64_t r0 = k0 + w;
    if (r0 >= n) break;
    const int64_t w2 = std::min<int64_t>(CH_NB, n - r0);
    // next block's columns (rectangle; its upper-triangle part is never read)
    gemm_nt_sub_launch(st, n - r0, w2, w, A + k0 * lda + r0, lda, A + k0 * lda + r0, lda, A + r0 * lda + r0, lda,
                       info);
    if (two) { hipEventRecord(ev_rel, st); hipStreamWaitEvent(side, ev_rel, 0); }
    if (n - r0 - w2 > 0) {
      GemmArgs a;
      a.ni = a.nj = n - r0 - w2;
      a.K = w;
      a.X = a.Y = A + k0 * lda + r0 + w2;
      a.ldx = a.ldy = lda;
      a.C = A + (r0 + w2) * lda + r0 + w2;
      a.ldc = lda;
      a.alpha = -1.0;
      a.beta = 1.0;
      a.info = info;
      a.tri = 1;
      // with the look-ahead running: persistent form on all but panel_reserve_cus() CUs, one
      // workgroup per CU, so the panel workgroups get CUs of their own (no fp64 MFMA neighbours)
      const int res = panel_reserve_cus();
      if (two && res > 0) mfma_gemm_launch_persistent(st, a, num_cus() - res);
      else mfma_gemm_launch(st, a);
    }
  }
  if (st != caller) { hipEventRecord(pst->ev_out, st); hipStreamWaitEvent(caller, pst->ev_out, 0); }
}

void potrf_lower(hipStream_t st, int64_t n, double* A, int64_t lda, int* info, double* ws) {
  potrf_lower_la(st, nullptr, n, A, lda, info, ws);
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

static void trsv_chain(hipStream_t st, bool fwd, int64_t n, const double* L, int64_t ldl, const double* b,
                       int64_t bstride, double* y, unsigned* ctl) {
  const int nblk = (int)cdiv(n, TV_B);
  const int grid = std::min(nblk, 1024);
  if (fwd)
    hipLaunchKernelGGL(k_trsv_chain<true>, dim3(grid), dim3(256), 0, st, n, nblk, L, ldl, b, bstride, y, ctl);
  else
    hipLaunchKernelGGL(k_trsv_chain<false>, dim3(grid), dim3(256), 0, st, n, nblk, L, ldl, b, bstride, y, ctl);
}

// L^T x = b (b read with stride bstride, e.g. the bordered row of a Cholesky factor); ctl: 2 words
void trsv_lower_t(hipStream_t st, int64_t n, const double* L, int64_t ldl, const double* b, int64_t bstride,
                  double* x, unsigned* ctl) {
  if (n <= 0) return;
  hipMemsetAsync(ctl, 0, 2 * sizeof(unsigned), st);
  trsv_chain(st, false, n, L, ldl, b, bstride, x, ctl);
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
                 int64_t ldb, double* W, unsigned* ctl) {
  if (n <= 0 || nrhs <= 0) return;
  if (nrhs == 1 && ldb == 1 && ctl) {
    hipMemsetAsync(ctl, 0, 4 * sizeof(unsigned), st);
    trsv_chain(st, true, n, L, ldl, B, 1, W, ctl);
    trsv_chain(st, false, n, L, ldl, W, 1, B, ctl + 2);
    return;
  }
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
