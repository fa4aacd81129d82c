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
// The eigendecomposition is rocSOLVER's dsyevd (a library call on the fallback path only: the
// Cholesky path never reaches it); both applications of V are rocBLAS dgemms on the same stream.
// Right-hand sides use the engine's row-major convention: B is n x nrhs, element (i, j) at
// B[i * ldb + j] -- i.e. B^T column-major with leading dimension ldb, so
//   X^T = B^T V diag(f) V^T  =  two GEMMs on B^T with a column scaling in between.
#include <hip/hip_runtime.h>
#include <rocblas/rocblas.h>
#include <rocsolver/rocsolver.h>

#include <cfloat>

#include "ipm_common.h"

namespace ipm {

// f_i = 1/lambda_i if |lambda_i| > eps * n * max|lambda| else 0 (syevd returns lambda ascending,
// so max|lambda| = max(|lambda_0|, |lambda_{n-1}|)).  f overwrites w.
__global__ void k_pinv_weights(int64_t n, double* __restrict__ w) {
  const double smax = fmax(fabs(w[0]), fabs(w[n - 1]));
  const double cut = DBL_EPSILON * (double)n * smax;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double l = w[i];
    w[i] = (fabs(l) > cut) ? 1.0 / l : 0.0;
  }
}

// C (column-major, rows x n, ld) column i *= f_i
__global__ void k_scale_cols(int64_t rows, int64_t n, double* __restrict__ C, int64_t ld,
                             const double* __restrict__ f) {
  const int64_t total = rows * n;
  for (int64_t e = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; e < total; e += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = e / rows, r = e - i * rows;
    C[i * ld + r] *= f[i];
  }
}

static rocblas_handle rb_get(void** slot, hipStream_t st) {
  if (!*slot) {
    rocblas_handle h = nullptr;
    if (rocblas_create_handle(&h) != rocblas_status_success) return nullptr;
    *slot = h;
  }
  rocblas_handle h = static_cast<rocblas_handle>(*slot);
  rocblas_set_stream(h, st);
  return h;
}

void lstsq_release(void* rb) {
  if (rb) rocblas_destroy_handle(static_cast<rocblas_handle>(rb));
}

int64_t lstsq_ws_doubles(int64_t n, int64_t nrhs) { return 2 * n + 64 + std::max<int64_t>(nrhs, 1) * n; }

// A (full symmetric, column-major, lda) -> eigenvectors V in place; ws[0:n] -> pseudo-inverse
// weights f.  info_dev (device int) = syevd's info (0 = converged).  Returns 0 or -1 (library error).
int lstsq_sym_factor(void** rb, hipStream_t st, int64_t n, double* A, int64_t lda, double* ws, int* info_dev) {
  if (n <= 0) return 0;
  rocblas_handle h = rb_get(rb, st);
  if (!h) return -1;
  double* w = ws;
  double* E = ws + n;
  if (rocsolver_dsyevd(h, rocblas_evect_original, rocblas_fill_lower, (rocblas_int)n, A, (rocblas_int)lda, w, E,
                       info_dev) != rocblas_status_success)
    return -1;
  k_pinv_weights<<<(unsigned)std::min<int64_t>((n + 255) / 256, 1024), 256, 0, st>>>(n, w);
  return 0;
}

// B (row-major n x nrhs, ldb) <- V diag(f) V^T B, with V, f from lstsq_sym_factor (same ws).
int lstsq_sym_apply(void** rb, hipStream_t st, int64_t n, int64_t nrhs, const double* V, int64_t ldv, double* B,
                    int64_t ldb, double* ws) {
  if (n <= 0 || nrhs <= 0) return 0;
  rocblas_handle h = rb_get(rb, st);
  if (!h) return -1;
  const double* f = ws;
  double* Ct = ws + 2 * n + 64;   // nrhs x n, column-major, ld nrhs
  const double one = 1.0, zero = 0.0;
  // C^T = B^T V
  if (rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_none, (rocblas_int)nrhs, (rocblas_int)n,
                    (rocblas_int)n, &one, B, (rocblas_int)ldb, V, (rocblas_int)ldv, &zero, Ct, (rocblas_int)nrhs) !=
      rocblas_status_success)
    return -1;
  const int64_t tot = nrhs * n;
  k_scale_cols<<<(unsigned)std::min<int64_t>((tot + 255) / 256, 4096), 256, 0, st>>>(nrhs, n, Ct, nrhs, f);
  // X^T = C^T V^T
  if (rocblas_dgemm(h, rocblas_operation_none, rocblas_operation_transpose, (rocblas_int)nrhs, (rocblas_int)n,
                    (rocblas_int)n, &one, Ct, (rocblas_int)nrhs, V, (rocblas_int)ldv, &zero, B, (rocblas_int)ldb) !=
      rocblas_status_success)
    return -1;
  return 0;
}

}  // namespace ipm
