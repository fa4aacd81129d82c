// Shared device helpers and launch-wrapper declarations for the ipm355 kernels.
// gfx950 only: wave64, fp64 MFMA (v_mfma_f64_16x16x4_f64).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

namespace ipm {

constexpr int WAVE = 64;

typedef double dbl4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// block-wide sum (blockDim.x multiple of 64, <= 1024); result valid in all threads
__device__ __forceinline__ double block_sum(double v, double* red /* >= 16 doubles LDS */) {
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6, nw = blockDim.x >> 6;
  v = wave_sum(v);
  __syncthreads();
  if (lane == 0) red[wid] = v;
  __syncthreads();
  double r = 0.0;
  for (int i = 0; i < nw; ++i) r += red[i];   // fixed order: deterministic
  return r;
}

// ---------------------------------------------------------------- launch wrappers
// dense kernels (ipm_blas.hip); all pointers are device pointers, fp64
// y[i] = alpha * sum_j M[i*ldm + j] x[j] + beta * y[i]        (rows x cols, row-major)
void gemv_n(hipStream_t s, int64_t rows, int64_t cols, double alpha, const double* M, int64_t ldm,
            const double* x, double beta, double* y);
// y[j] = alpha * sum_i w[i] M[i*ldm + j] x[i] + beta * y[j]   (w may be null)
void gemv_t(hipStream_t s, int64_t rows, int64_t cols, double alpha, const double* M, int64_t ldm,
            const double* x, const double* w, double beta, double* y, double* partial_ws,
            int64_t partial_ws_elems);
int64_t gemv_t_ws_elems(int64_t rows, int64_t cols);
// y1 = M1 x, y2 = M2 x in one launch (bitwise gemv_n's rows; two launches if the alignments differ)
void gemv_n2(hipStream_t s, int64_t cols, const double* x, int64_t r1, const double* M1, int64_t ld1, double* y1,
             int64_t r2, const double* M2, int64_t ld2, double* y2);
// ct = M^T x (gemv_t with alpha 1, beta 0, no weights) and g = the barrier gradient combine of
// (go, blb, bub, ct) in the same launch as the column sums (bitwise gemv_t + grad_combine)
void gemv_t_grad(hipStream_t s, int64_t rows, int64_t cols, const double* M, int64_t ldm, const double* x,
                 double* ct, double* part, int64_t part_elems, const double* go, const double* blb,
                 const double* bub, bool ct_first, double* g);

// lower triangle (column-major, ldh) of  H = alpha * X^T diag(w) Y + beta * H + tP * P + diag(dvec)
// X, Y row-major k x n (ld ldx, ldy).  w, P, dvec may be null.  Y may equal X.
struct SyrkEpi {
  const double* P = nullptr;   // row-major symmetric, ldp
  int64_t ldp = 0;
  double tP = 0.0;
  const double* dvec = nullptr;
  // split tail (k_mfma_gemm_split): split_cap partial tiles of 128 x 128, then split_cap flags;
  // null: the plain tile grid
  double* split_ws = nullptr;
  int64_t split_cap = 0;
  // the flag area is zero on entry (zeroed once when the workspace was carved): the kernels leave
  // it zero (the last piece / the consuming K half resets its word), so no memset per call
  bool flags_zero = false;
};
// workspace of the split tail for an n x n lower-triangle SYRK: the cap and its size in doubles
inline int64_t syrk_split_cap(int64_t n) {
  const int64_t T = (n + 63) / 64;   // 64-tile grid (the launcher uses 64-tiles below 768 128-tiles)
  return std::min<int64_t>(256, std::max<int64_t>(T * (T + 1) / 2, 8));
}
// (flag area: 2c + 4 words -- the stream-K tail's tile counters and per-piece words)
inline int64_t syrk_split_ws_doubles(int64_t n) {
  const int64_t c = syrk_split_cap(n);
  return c * 128 * 128 + c + 2;
}
void syrk_lower(hipStream_t s, int64_t n, int64_t k, double alpha, const double* X, int64_t ldx,
                const double* Y, int64_t ldy, const double* w, double beta, double* H, int64_t ldh,
                const SyrkEpi& epi);
// C(m x n, column-major ldc) -= A(m x k, col-major lda) * B(n x k, col-major ldb)^T
//   (the GEMM of the Cholesky panel / trailing update, general rectangle)
void gemm_nt_sub(hipStream_t s, int64_t m, int64_t n, int64_t k, const double* A, int64_t lda,
                 const double* B, int64_t ldb, double* C, int64_t ldc);
// C(i, j) = sum_k X[k][i] Y[k][j] over the FULL ni x nj rectangle (column-major C, ldc; X, Y
// k-major): a product whose two triangles are computed separately, e.g. the non-symmetric
// S = A (H^-1 A^T) of the infeasible-start block elimination
void gemm_kk(hipStream_t s, int64_t ni, int64_t nj, int64_t k, const double* X, int64_t ldx, const double* Y,
             int64_t ldy, double* C, int64_t ldc);

// Cholesky (column-major lower, in place). info_dev: device int (0 or first failing column, 1-based)
// ws: device workspace of potrf_ws_doubles(n) doubles: two panels' inverted diagonal blocks and
// published L11 blocks, then the control words (per launch: a header, one word per 64-row block
// for the look-ahead tiles and one per 64-row chunk of the first panel)
// trailing tiles a launch may split in two K halves (its last round): flags in the control
// words, one 128 x 128 partial tile each in the workspace
__host__ __device__ inline int64_t potrf_split_cap(int64_t n) {
  const int64_t t = (n + 127) / 128, tri = t * (t + 1) / 2;
  return tri < 512 ? tri : 512;
}
__host__ __device__ inline int64_t block_ctl_words(int64_t n) {
  return 64 + 2 * ((n + 63) / 64) + 8 + potrf_split_cap(n);   // (header: CTL_HDR <= 64 words)
}
inline int64_t potrf_split_scratch_off(int64_t n) {
  return ((2 * (8 * 256 + 36 * 256) + (8 + ((n + 127) / 128) * block_ctl_words(n) + 1) / 2 + 8) + 31) & ~int64_t(31);
}
inline int64_t potrf_ws_doubles(int64_t n) { return potrf_split_scratch_off(n) + potrf_split_cap(n) * 128 * 128; }
void potrf_lower(hipStream_t s, int64_t n, double* H, int64_t ldh, int* info_dev, double* ws);

// Blocked right-looking Cholesky, one launch per 256-column block on stream s (k_potrf_block).
// ncols < n: only the first ncols columns are factored (all n rows) -- the bordered Newton system
// needs row n-1 of L (the forward-solved right-hand side) but not its diagonal entry.
// the bordered right-hand side (border_rhs's row N = scale * g, corner) written by the launch
// that zeroes the control words (one launch fewer per Newton step)
struct BorderJob {
  int64_t N = 0, ldh = 0;
  double* H = nullptr;
  const double* g = nullptr;
  double scale = -1.0, corner = 1e300;
};
void potrf_lower_fused(hipStream_t s, int64_t n, double* H, int64_t ldh, int* info_dev, double* ws,
                       int64_t ncols = -1, const BorderJob* border = nullptr);
// L L^T X = B in place, L column-major lower; B row-major n x nrhs (ldb); W scratch n x nrhs;
// ctl: 4 device words for the single-RHS persistent solves (null -> blocked multi-RHS path)
void potrs_lower(hipStream_t s, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B,
                 int64_t ldb, double* W, unsigned* ctl, double* xinv_ws = nullptr, unsigned* err = nullptr);
// L L^T X = B for many right-hand sides (nrhs >~ 32): 128-row blocks on MFMA GEMMs; ws of
// potrs_blocked_ws_doubles(n, nrhs) doubles
int64_t potrs_blocked_ws_doubles(int64_t n, int64_t nrhs);
void potrs_blocked(hipStream_t s, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B, int64_t ldb,
                   double* ws);
// L^T x = b, one right-hand side read with stride bstride; ctl: 2 device words
// xinv_ws: trsv_inv_ws_doubles(n) doubles for the inverted 128 x 128 diagonal blocks; err: sticky
// device error word (bit 0: a chain producer missed the spin bound; the caller must read it before
// using x).  Either null: the 64-row substitution kernel (unbounded waits, no error word).
// b must not contain the all-ones NaN bit pattern (the persistent solve's "pending" marker).
void trsv_lower_t(hipStream_t s, int64_t n, const double* L, int64_t ldl, const double* b, int64_t bstride,
                  double* x, unsigned* ctl, double* xinv_ws = nullptr, unsigned* err = nullptr);
// spin bound (sleeps) of the backward solve's chain poll; 0 restores the default 2^20 (debug knob:
// ipm_debug_set_trsv_spin_limit)
void set_trsv_spin_limit(unsigned lim);
// bound (microseconds of wall clock, 0 = default 1 s) of every wait inside the ticketed Cholesky
// (debug knob: ipm_debug_set_potrf_spin_limit); a missed bound makes *info = POTRF_INFO_SPIN (-1000)
void set_potrf_spin_limit_us(unsigned us);
constexpr int POTRF_INFO_SPIN = -1000;
// debug knob: the k-th lstsq_sym_factor call from now reports non-convergence (-1: off)
void set_lstsq_fail_call(int k);
// debug knob: the workgroup holding this ticket of the backward solve sleeps ~7 ms before it
// publishes its progress word (-1: none)
void set_trsv_publish_delay(int ticket);
inline int64_t trsv_inv_ws_doubles(int64_t n) { return ((n + 127) / 128) * 128 * 128; }
// H[j*ldh + N] = scale * g[j] (j < N), H[N*ldh + N] = 1e300: bordered right-hand side (see ipm_blas.hip)
void border_rhs(hipStream_t s, int64_t N, double* H, int64_t ldh, const double* g, double scale);
// forward L Y = B / backward L^T Y = B: B is consumed, the solution goes to Y (same ld)
void trsm_lower_fwd(hipStream_t s, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B,
                    int64_t ldb, double* Y);
void trsm_lower_bwd(hipStream_t s, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B,
                    int64_t ldb, double* Y);
// LU with partial pivoting (row-major in/out copy in column-major work), solve; used as the
// Cholesky fallback (NewtonSolver.py:334-341, NewtonSolverInfeasibleStart.py:513-538)
// ws: LU_NB * n doubles (the U12 panel operand of the trailing GEMM)
void getrf(hipStream_t s, int64_t n, double* A, int64_t lda, int64_t* piv, int* info_dev, double* ws);
inline int64_t getrf_ws_doubles(int64_t n) { return 64 * (n + 1); }
void getrs(hipStream_t s, int64_t n, int64_t nrhs, const double* LU, int64_t lda, const int64_t* piv,
           double* B, int64_t ldb);
// minimum-norm least squares on a symmetric matrix, np.linalg.lstsq(H, B, rcond=None) (ipm_lstsq.hip):
// factor = eigendecomposition (A full column-major; ws <- the eigenvectors V and the pseudo-inverse
// weights, A <- V^T), apply = B (row-major n x nrhs) <- H^+ B (W = the factored A).  The blocked
// Jacobi above n = 256 does one 4-byte readback per sweep.  rb: lazily created library
// handle slot.  ws: lstsq_ws_doubles(n, nrhs) doubles.  Return 0, or -1 on a library error.
// *info_dev is STICKY: the factor sets it to 1 on non-convergence and never clears it (the caller
// zeroes it once before a group of factorizations and reads it after all of them).
int64_t lstsq_ws_doubles(int64_t n, int64_t nrhs);
int lstsq_sym_factor(void** rb, hipStream_t s, int64_t n, double* A, int64_t lda, double* ws, int* info_dev);
int lstsq_sym_apply(void** rb, hipStream_t s, int64_t n, int64_t nrhs, const double* W, int64_t ldw, double* B,
                    int64_t ldb, double* ws);
// column-major lower triangle -> full symmetric, in place (the upper triangle is overwritten)
void sym_expand_inplace(hipStream_t s, int64_t n, double* M, int64_t ld);
void lstsq_release(void* rb);

// small helpers
void fill(hipStream_t s, double* p, int64_t n, double v);
void copy(hipStream_t s, double* dst, const double* src, int64_t n);
// dst(col-major lower, ldd) full symmetric expansion into row-major full out (ldo)
void sym_lower_to_full(hipStream_t s, int64_t n, const double* L, int64_t ldl, double* out, int64_t ldo);
void transpose(hipStream_t s, int64_t rows, int64_t cols, const double* in, int64_t ldi, double* out,
               int64_t ldo);

}  // namespace ipm
