/*
 * ipm355.h -- C ABI of the MI355X (gfx950) interior-point Newton hot path.
 *
 * Drop-in boundary for the reference's Newton inner loop
 * (fdeguire03/InteriorPoint-GPU).  The reference is pure Python with no FFI;
 * its seam between the problem facades (LPSolver/QPSolver/SOCPSolver) and the
 * numerics is the "oracle protocol" of FunctionManager.py:94-195 and the
 * Newton protocol of NewtonSolver.py:80 / NewtonSolverInfeasibleStart.py:72.
 * Each entry point below names the reference interface it replaces.
 * The Python binding (ctypes) lives in interiorpoint-gpu_amd/ipm355/_lib.py;
 * INTEGRATION.md shows the stub a reference maintainer would add.
 *
 * Conventions
 *   - fp64 everywhere.  Dense inputs are row-major (C order) with explicit
 *     leading dimensions, exactly as NumPy hands them over.
 *   - Every pointer argument marked [dev] is a device pointer (in practice a
 *     torch tensor's data_ptr()); the library never allocates device memory on
 *     the hot path: the caller provides a workspace of ipm_workspace_bytes().
 *   - All work is enqueued on the handle's stream.  Entry points that return
 *     host scalars synchronise that stream once.
 *   - Return value: IPM_OK or an error code; ipm_last_error() has the text.
 */
#ifndef IPM355_H
#define IPM355_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define IPM_OK 0
#define IPM_NOT_POSITIVE_DEFINITE 1 /* LAPACK potrf info > 0 (drives Q9 fallback) */
#define IPM_INVALID_ARG 2
#define IPM_HIP_ERROR 3
#define IPM_NOT_SUPPORTED 4
#define IPM_LINALG_NOT_CONVERGED 5 /* the least-squares eigensolver did not converge (numpy: LinAlgError
                                      "SVD did not converge in Linear Least Squares") */

/* problem kinds (LPSolver.py / QPSolver.py / SOCPSolver.py) */
#define IPM_KIND_LP 0
#define IPM_KIND_QP 1
#define IPM_KIND_SOCP 2

/* linear-solve strategies (dispatch tables LPSolver.py:371-469, QPSolver.py:385-455) */
#define IPM_SOLVE_CHOLESKY 0 /* dense Cholesky; first failure -> permanent fallback (Q9) */
#define IPM_SOLVE_DIAGONAL 1 /* H diagonal (LP, C is None, try_diag) */
#define IPM_SOLVE_LU 2       /* np_solve / direct: LU with partial pivoting */
#define IPM_SOLVE_LSTSQ 3    /* np_lstsq: minimum-norm least squares (lstsq(H, -g, rcond=None)) */
#define IPM_SOLVE_DIAGONAL_LSTSQ 4 /* diagonal H, equality system S = A H^-1 A^T by lstsq
                                      (NewtonSolverNPLstSqDiagonalInfeasibleStart) */

typedef struct ipm_handle ipm_handle;
typedef struct ipm_problem ipm_problem;

/*
 * Problem description.  Mirrors the data the reference's FunctionManager*
 * constructors receive (FunctionManager.py:13-90, 359-425, 619-680, 834-931,
 * 1165-1256).  Absent items are NULL.  Scalar bounds are expanded to n-vectors
 * by the caller.
 */
typedef struct ipm_problem_desc {
  int32_t kind;          /* IPM_KIND_*                                           */
  int32_t phase1;        /* 1: the phase-1 barrier (FunctionManagerPhase1 /      */
                         /*    FunctionManagerSOCPPhase1); variables (x, s)      */
  int32_t solve_method;  /* IPM_SOLVE_*                                          */
  int32_t reserved0;
  int64_t n;             /* number of x variables (without the phase-1 s)        */
  /* objective */
  const double* c;       /* [dev] n      LP cost (FunctionManager.py:76-90)       */
  const double* P;       /* [dev] n x n  QP/SOCP quadratic term, row-major        */
  int64_t ldp;
  const double* q;       /* [dev] n      QP/SOCP linear term                      */
  /* linear inequalities C x <= d (LP, QP, LP phase 1) */
  int64_t m;
  const double* C;       /* [dev] m x n  row-major                                */
  int64_t ldc;
  const double* d;       /* [dev] m                                               */
  /* box bounds */
  const double* lb;      /* [dev] n                                               */
  const double* ub;      /* [dev] n                                               */
  /* equality constraints A x = b -> infeasible-start Newton
     (NewtonSolverInfeasibleStart.py; SOCPSolver passes F, g here)               */
  int64_t p;
  const double* A;       /* [dev] p x n  row-major                                */
  int64_t lda;
  const double* AT;      /* [dev] n x p  row-major copy of A^T (static, once)     */
  const double* b;       /* [dev] p                                               */
  /* second-order cones (FunctionManagerSOCP): ||A_i x + b_i|| <= c_i.x + d_i    */
  int64_t K;             /* number of cones                                       */
  int64_t R;             /* total rows of the dense cones                         */
  double* X;             /* [dev] (R + 2K) x n row-major, ldx: rows [0,R) stacked */
                         /*   dense A_i, rows [R,R+K) the c_i, rows [R+K,R+2K)    */
                         /*   scratch for the per-cone gradient rows g_i          */
  int64_t ldx;
  const int64_t* cone_row_off; /* [dev] K+1: rows of cone i are [off[i],off[i+1]); */
                               /*   a diagonal cone has off[i]==off[i+1]           */
  const int64_t* cone_row_off_host; /* host copy of the above                     */
  const double* cone_b;  /* [dev] R: b_i stacked for the dense rows (NULL: no b)   */
  const double* cone_d;  /* [dev] K: d_i (NULL: no d)                              */
  int32_t has_cone_c;    /* 0: no c_i (rhs_i = d_i)                                */
  int32_t reserved1;
  int64_t Kd;            /* number of diagonal cones (A_i = diag(a_i), SOCPSolver.py:285-292) */
  const double* Ad;      /* [dev] Kd x n  a_i                                       */
  const double* bd;      /* [dev] Kd x n  b_i (NULL: no b)                          */
  const int64_t* dcone_id; /* [dev] Kd: cone index of each diagonal cone            */
  const int64_t* dcone_id_host;
} ipm_problem_desc;

/* Newton options: NewtonSolver.__init__ (NewtonSolver.py:16-78) */
typedef struct ipm_newton_opts {
  int32_t max_iters;
  int32_t update_slacks_every;   /* Q2 */
  int32_t phase1_flag;           /* early exit x[-1] < -phase1_tol (NewtonSolver.py:105-107) */
  int32_t use_psd_condition;     /* +1e-9 on diag before Cholesky (NewtonSolver.py:269-275) */
  double eps;                    /* inner epsilon */
  double alpha, beta;            /* backtracking parameters */
  double phase1_tol;
  double* trace;                 /* optional HOST buffer: per-iteration (step, stat) pairs  */
  int32_t trace_cap;             /* capacity in iterations (0: no trace)                   */
  int32_t linesearch_mode;       /* IPM_LS_* (feasible start)                                */
} ipm_newton_opts;

/* feasible-start backtracking (NewtonSolver.py:157-206) */
#define IPM_LS_TABLE 0   /* 64 candidate steps per pass: slacks s0 + a ds, f(x + a dx) by its
                            expansion; the reference's decision sequence replayed on the host   */
#define IPM_LS_EXACT 1   /* reference-exact: every trial point formed, fresh d - C next_x slacks
                            when the reference refreshes them, f(next_x) evaluated directly      */
#define IPM_LS_COMPARE 2 /* both; the exact step is taken, disagreements counted (ls_flips)     */

/* Result of one centering step: the tuple NewtonSolver.solve returns */
typedef struct ipm_newton_result {
  int32_t iters;        /* Newton iterations taken                               */
  int32_t success;      /* success flag                                          */
  int32_t stat_valid;   /* 0: the reference would return None                    */
  int32_t use_backup;   /* Cholesky fallback engaged (persists, Q9)              */
  double stat;          /* nd = -g.dx/2 (feasible) or trial residual (infeasible)*/
  double last_step;     /* last accepted step size                               */
  int64_t backtracks;   /* total trial points examined                           */
  int64_t ls_compared;  /* IPM_LS_COMPARE: steps compared / steps whose table and  */
  int64_t ls_flips;     /*   exact step sizes differ                             */
  int64_t linalg_error; /* the solve ended on a LinAlgError: a least-squares      */
                        /*   eigensolve did not converge (the reference's try /   */
                        /*   except in NewtonSolver.py:148-155 returns a failure)  */
} ipm_newton_result;

/* ---- handle --------------------------------------------------------------- */
/* one handle per (process, device, stream); stream = hipStream_t, NULL = legacy default stream */
int ipm_create(int device, void* stream, ipm_handle** out);
int ipm_destroy(ipm_handle* h);
const char* ipm_last_error(ipm_handle* h);
int ipm_version(void);

/* ---- level 2: the Newton inner loop (the hot path) ------------------------- */
/* bytes of device workspace the problem needs */
int64_t ipm_workspace_bytes(const ipm_problem_desc* desc);
int ipm_problem_create(ipm_handle* h, const ipm_problem_desc* desc, void* workspace /*[dev]*/,
                       int64_t workspace_bytes, ipm_problem** out);
int ipm_problem_destroy(ipm_problem* pr);
/* NewtonSolver.solve / NewtonSolverInfeasibleStart.solve: x [dev] (N = n(+1)) is
   updated in place (Q8); v [dev] (p) likewise; t is the barrier parameter. */
int ipm_newton_solve(ipm_problem* pr, double* x, double t, double* v, const ipm_newton_opts* opts,
                     ipm_newton_result* res);
/* persistent Cholesky-failure flag (Q9) */
int ipm_get_use_backup(ipm_problem* pr);
int ipm_set_use_backup(ipm_problem* pr, int flag);

/* ---- level 1: the oracle protocol (FunctionManager.py:94-195) ---------------- */
/* update_x(x, update_slacks): the evaluation point becomes x [dev]; slacks are
   recomputed only if update_slacks (Q2) */
int ipm_fm_update_x(ipm_problem* pr, const double* x, int update_slacks);
/* slacks [dev out] (FunctionManager.slacks) */
int ipm_fm_slacks(ipm_problem* pr, double* out);
int64_t ipm_fm_num_slacks(ipm_problem* pr);
/* objective(): f(x) at the evaluation point (host scalar) */
int ipm_fm_objective(ipm_problem* pr, double* out);
/* newton_objective(): t f(x) - sum log(s + eps) with the CURRENT (maybe stale) slacks */
int ipm_fm_newton_objective(ipm_problem* pr, double t, double* out);
/* gradient() [dev out, N] */
int ipm_fm_gradient(ipm_problem* pr, double t, double* g);
/* hessian() [dev out]: dense N x N row-major full matrix (both triangles), or for
   IPM_SOLVE_DIAGONAL the diagonal vector (N) */
int ipm_fm_hessian(ipm_problem* pr, double t, double* H, int64_t ldh);

/* ---- level 0: dense fp64 kernels (exposed for tests and benches) -------------- */
/* y = alpha * op(M) x + beta * y ; M row-major rows x cols */
int ipm_gemv(ipm_handle* h, int trans, int64_t rows, int64_t cols, double alpha, const double* M,
             int64_t ldm, const double* x, double beta, double* y);
/* H(lower, column-major ldh) = alpha * X^T diag(w) X + beta * H ; X row-major k x n.
   w may be NULL (all ones).  The SYRK of FunctionManager.py:301-306 / 801-805. */
int ipm_syrk(ipm_handle* h, int64_t n, int64_t k, const double* X, int64_t ldx, const double* w,
             double alpha, double beta, double* H, int64_t ldh);
/* in-place Cholesky of the lower triangle of H (column-major, ldh); *info as LAPACK
   potrf (0 ok, j>0: leading minor j not positive definite).  work: [dev] >= 64 bytes */
int ipm_potrf(ipm_handle* h, int64_t n, double* H, int64_t ldh, int* info);
/* the first ncols columns only (0 <= ncols <= n): L11 = chol(H11) and L21 = H21 L11^-T, the
   rows below ncols untouched otherwise.  The Newton step factors [[H, -g], [-g^T, .]] this way
   with ncols = N, so row N becomes L^-1 (-g): the forward substitution of cho_solve
   (NewtonSolver.py:303-313) rides inside the factorisation */
int ipm_potrf_partial(ipm_handle* h, int64_t n, int64_t ncols, double* H, int64_t ldh, int* info);
/* solve L L^T X = B in place; L lower column-major (ldl); B row-major n x nrhs (ldb) */
int ipm_potrs(ipm_handle* h, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B,
              int64_t ldb);
/* LU with partial pivoting, in place (column-major, lda): the np.linalg.solve / Cholesky-fallback
   factorisation (NewtonSolver.py:230-247, 334-341; NewtonSolverInfeasibleStart.py:513-538).  Blocked:
   64-column panels, MFMA trailing update.  piv [dev] n: row swapped with k, or -1-k for an exactly
   zero pivot column (skipped; ipm_getrs gives that component 0) */
int ipm_getrf(ipm_handle* h, int64_t n, double* A, int64_t lda, int64_t* piv, int* info);
/* solve with the ipm_getrf factors; B row-major n x nrhs (ldb), in place */
int ipm_getrs(ipm_handle* h, int64_t n, int64_t nrhs, const double* LU, int64_t lda, const int64_t* piv,
              double* B, int64_t ldb);
/* minimum-norm least squares on a symmetric matrix: B <- A^+ B, the np.linalg.lstsq(A, B, rcond=None)
   of the np_lstsq method and of the Cholesky-failure backup (NewtonSolver.py:212-227, 334-341;
   NewtonSolverInfeasibleStart.py:279-316, 692-724).  A full symmetric (column-major, lda), replaced
   by W = V^T, the TRANSPOSED eigenvector matrix (column-major, lda: column j of A holds row j of V,
   i.e. A(i, j) = V(j, i), the operand layout of the MFMA apply); eigenvalues
   |lambda| <= eps * n * max|lambda| are dropped (gelsd's rcond rule).  B row-major n x nrhs (ldb), in place.  *info: the eigensolver's convergence info (0 = ok,
   1 = the hand-written Jacobi eigensolver did not converge) */
int ipm_lstsq_sym(ipm_handle* h, int64_t n, int64_t nrhs, double* A, int64_t lda, double* B, int64_t ldb,
                  int* info);
/* HIP-event timing of the KKT assembly and of the Cholesky factorisation inside
   ipm_newton_solve (enable/reset with ipm_set_timing; adds no synchronisation):
   averages (ms) over the Newton iterations since the reset, and their count */
int ipm_set_timing(ipm_handle* h, int on);
int ipm_last_timings(ipm_handle* h, double* kkt_ms, double* potrf_ms, double* count);
/* debug knob: the wall-clock bound (microseconds, s_memrealtime) after which the persistent
   backward solve's chain step stops waiting for its producer and raises its device error word; the
   Newton step's readback then returns IPM_HIP_ERROR instead of using the step.  0 restores the
   default 1 s.  Process-wide; tests use a tiny bound to trip the error path once. */
int ipm_debug_set_trsv_spin_limit(unsigned limit);
/* debug knob: the same wall-clock bound (microseconds; 0 = default 1 s) for every wait of the
   ticketed Cholesky (k_potrf_block: row chunks on their diagonal role, look-ahead / fold / split
   hand-offs, trailing tiles kept off critical CUs).  A wait that runs out sets info to -1000
   (IPM_INFO_SPIN: never a LAPACK column), every later launch of the factorization returns at once,
   and ipm_potrf / the Newton step return IPM_HIP_ERROR.  Process-wide. */
int ipm_debug_set_potrf_spin_limit(unsigned microseconds);
/* debug knob: the k-th least-squares eigensolve from now (k = 0: the next one) reports
   non-convergence whatever happened (-1: off).  Tests that one failed eigensolve among several in
   a Newton step is not overwritten by a later converged one. */
int ipm_debug_lstsq_fail_call(int k);
/* debug knob: the backward-solve workgroup holding chain ticket `ticket` sleeps ~7 ms before
   publishing its progress word (-1: off), so later tickets overtake it -- exercises the monotonic
   progress publish.  ticket <= -2: ticket -2 - ticket sleeps before storing its x block instead,
   so the next ticket's bounded poll of that block runs out (exercises the loud failure).
   Process-wide. */
int ipm_debug_set_trsv_publish_delay(int ticket);
/* KKT-SYRK flops of one Newton step of this problem (m n (n+1) in total): all of them run in the
   SYRK kernel (*upfront); *deferred is always 0 (the round-2 deferred-slice experiment was
   removed; the argument is kept so existing bindings need no change) */
int ipm_kkt_flops(ipm_problem* pr, double* upfront, double* deferred);
/* measurement: HIP-event time (ms, averaged over `reps`, on the handle's stream) of the HBM-bound
   kernels of one Newton step on this problem's buffers -- ms[0] the slack GEMV C x, ms[1] the
   gradient GEMV C^T w, ms[2] one 64-candidate line-search pass over the S slacks.  Clobbers only
   scratch.  LP/QP problems with inequality rows (bench.py reports them as GB/s). */
int ipm_time_hbm_kernels(ipm_problem* pr, int reps, double* ms);
/* out[0..2] = m (inequality rows), n, S (slacks incl. box bounds) */
int ipm_problem_sizes(ipm_problem* pr, int64_t* out);

/* ---- batched ADMM Lasso (LassoSolver.py) ------------------------------ *
 * S problems  min_x 1/(2m) ||A x - b_s||^2 + reg_s ||x||_1  solved together.  Every n x S matrix
 * below is row-major with leading dimension lds (element (i, s) at i*lds + s).                  */
typedef struct ipm_lasso_args {
  int64_t n, S, m;         /* variables (incl. the bias column), problems, rows of A           */
  int64_t lds;             /* leading dimension of x, alpha, u, W0, W1                         */
  const double* Qs;        /* [dev] n x n, ldq: (-m rho Q)^T, Q = (diag(m rho) + A^T A)^-1      */
  int64_t ldq;
  const double* bA;        /* [dev] n x (S or 1), ldba: Q A^T b (LassoSolver.py:214-219)         */
  int64_t ldba;
  const double* eta;       /* [dev] S or 1: reg / rho                                         */
  double* x;               /* [dev] state (zeros on entry, LassoSolver.py:222-236)             */
  double* alpha;
  double* u;
  double* W0;              /* [dev] u - alpha on entry; W1 scratch (ping-pong)                 */
  double* W1;
  double* partial;         /* [dev] >= ipm_lasso_partial_doubles(n, S), zeroed once before use  */
  double rho, eps_abs, eps_rel, stop_multiplier;
  int32_t max_iters, check_stop;
  int32_t positive, add_bias;
  int32_t dual_form;       /* 0: u = u + x - alpha (:251); 1: u = u + (x - alpha) (chunks, :413) */
  int32_t compute_loss;    /* per-iteration loss into gaps (LassoSolver.py:254-268)            */
  int32_t ba_bcast, eta_bcast, b_bcast, reg_bcast;   /* 1: a single column / value for all S   */
  /* loss evaluation (compute_loss, ipm_lasso_loss) */
  const double* AT;        /* [dev] n x m, ldat: A^T row-major                                 */
  int64_t ldat;
  const double* b;         /* [dev] m x (S or 1), ldb                                          */
  int64_t ldb;
  const double* reg;       /* [dev] S or 1                                                    */
  double* R;               /* [dev] m x S scratch                                             */
  double* gaps;            /* [dev] max_iters rows of ldg: gaps[it*ldg + col(s)]               */
  int64_t ldg;
  const int64_t* gap_cols; /* [dev] S: column of problem s in gaps (chunks), NULL: s            */
  int32_t qs_blocked;      /* 1: Qs is the tile-blocked copy of ipm_lasso_block_qs (ldq unused)  */
} ipm_lasso_args;

/* row-major C (M x N, ldc) = alpha A^T B + beta C; A: K x M (lda), B: K x N (ldb); fp64 MFMA */
int ipm_gemm_tn(ipm_handle* h, int64_t M, int64_t N, int64_t K, double alpha, const double* A, int64_t lda,
                const double* B, int64_t ldb, double beta, double* C, int64_t ldc);
/* out (cols x rows, ldo) = in^T (rows x cols, ldi), row-major; device copy of n doubles */
int ipm_transpose(ipm_handle* h, int64_t rows, int64_t cols, const double* in, int64_t ldi, double* out,
                  int64_t ldo);
int ipm_copy(ipm_handle* h, double* dst, const double* src, int64_t n);
/* normalize_A (LassoSolver.py:122-123): A /= A.std(axis=0) in place; stdv [dev] n (may be NULL) */
int ipm_lasso_colnorm(ipm_handle* h, int64_t m, int64_t n, double* A, int64_t lda, double* stdv);
/* add_bias (LassoSolver.py:124-131): out (m x (n+1), ldo) = [1 | A] */
int ipm_lasso_bias(ipm_handle* h, int64_t m, int64_t n, const double* A, int64_t lda, double* out, int64_t ldo);
/* LassoSolver.py:157-189: Q = (diag(m rho) + A^T A)^-1 via Cholesky (info as ipm_potrf), QT = Q^T */
int ipm_lasso_qinv(ipm_handle* h, int64_t m, int64_t n, const double* A, int64_t lda, double rho, double* Q,
                   double* QT, int64_t ldq, int* info);
/* M (rows x cols, ld) *= f1 (then *= f2 when two): Qinv *= -m*rho, or Qinv * -m * rho (chunks) */
int ipm_lasso_scale(ipm_handle* h, int64_t rows, int64_t cols, double* M, int64_t ld, double f1, double f2,
                    int two);
/* prox (LassoSolver.py:533-558): out = soft-threshold(v, eta), row 0 kept with add_bias */
int ipm_lasso_prox(ipm_handle* h, int64_t n, int64_t S, const double* v, int64_t ldv, const double* eta,
                   int eta_bcast, int positive, int add_bias, double* out, int64_t ldo);
/* loss per problem of the current alpha into out[cols ? cols[s] : s]; absm: |alpha| in the l1 term */
int ipm_lasso_loss(ipm_handle* h, const ipm_lasso_args* a, int absm, double* out, const int64_t* cols);
int64_t ipm_lasso_partial_doubles(int64_t n, int64_t S);
/* Qs (n x n, ldq, k-major) -> Qb in the ADMM step's tile-blocked layout: 32-row tiles of i, each
   tile's k rows contiguous (element (i, k) at ((i / 32) * n + k) * 32 + i % 32, rows >= n zero), so
   that each workgroup of the iteration GEMM streams one contiguous span instead of 256-byte pieces
   of every k row.  Qb holds ipm_lasso_qb_doubles(n) doubles. */
int64_t ipm_lasso_qb_doubles(int64_t n);
int ipm_lasso_block_qs(ipm_handle* h, int64_t n, const double* Qs, int64_t ldq, double* Qb);
/* the ADMM loop (LassoSolver.py:240-337, one chunk of :339-485): iterates until the stopping
   test (every check_stop iterations) or max_iters; *iters = the last iteration index */
int ipm_lasso_admm(ipm_handle* h, const ipm_lasso_args* a, int32_t* iters);

#ifdef __cplusplus
}
#endif
#endif /* IPM355_H */
