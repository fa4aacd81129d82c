// Barrier-oracle / line-search kernel declarations (ipm_barrier.hip).
#pragma once
#include "ipm_common.h"

namespace ipm {

// SOCP structure on device (see ipm_problem_desc in include/ipm355.h)
struct SocpView {
  int64_t n, K, R, Kd, nbnd;       // nbnd = n*(has_ub) + n*(has_lb)
  double* X;                       // (R + 2K) x n, ldx
  int64_t ldx;
  const int64_t* off;              // K+1 dense-row offsets
  const int64_t* rowcone;          // R: cone of each dense row
  const int64_t* dslot;            // K: diagonal-cone slot or -1
  const double* cb;                // R or null
  const double* cd;                // K or null
  int has_c;
  const double* Ad;                // Kd x n
  const double* bd;                // Kd x n or null
};

// infeasible-start residual candidate inputs
struct ResidView {
  int64_t n, p;
  double t;
  const double* c;                 // LP cost (then P terms unused) or null
  const double* Px;                // P x or null
  const double* Pdx;               // P dx or null
  const double* q;                 // or null
  const double* B;                 // barrier gradient at the (stale) slacks (used when blb, bub, ct all null)
  // the barrier gradient's pieces at the (stale) slacks, combined with the objective gradient in
  // the reference's own order (FunctionManager.py:248-263: grad = t c; -= 1/s_lb; += 1/s_ub;
  // += C^T 1/s; SOCP ct_first :1080-1100): at large t the terms cancel to a residual near the
  // rounding floor, so the association decides whether the backtracking test passes
  const double* blb = nullptr;
  const double* bub = nullptr;
  const double* ct = nullptr;
  bool ct_first = false;
  const double* ATv;
  const double* ATdv;
  const double* Axb;
  const double* Adx;
};

enum RedKind { RED_DOT = 0, RED_SUM = 1, RED_SUMSQ = 2, RED_SUMLOG = 3, RED_SUMINV = 4, RED_SUMINV2 = 5 };
struct ReduceOp {
  const double* a;
  const double* b;
  int64_t len, sa, sb;
  int kind, slot;
};
constexpr int MAX_RED = 24;
struct ReduceBatch {
  ReduceOp ops[MAX_RED];
};

void slacks_lin(hipStream_t st, int64_t n, int64_t m, const double* d, const double* Cx, const double* lb,
                const double* ub, const double* x, const double* shp, double* s);
void inv_eps(hipStream_t st, int64_t len, const double* s, double eps, double* out);
void square(hipStream_t st, int64_t len, const double* a, double* out);
void objgrad(hipStream_t st, int64_t n, double t, const double* c, const double* Px, const double* q,
             double* go);
void grad_combine(hipStream_t st, int64_t n, const double* go, const double* blb, const double* bub,
                  const double* ct, bool ct_first, double* g);
void dvec_sq(hipStream_t st, int64_t n, const double* a, const double* b, double add, double* out);
void dvec_inv_sq(hipStream_t st, int64_t n, const double* slb, const double* sub, double add, double* out);
void dvec_inv_eps_sq(hipStream_t st, int64_t n, const double* slb, const double* sub, double add, double* out);
void dvec_diag_cones(hipStream_t st, int64_t n, int64_t Kd, const double* Ad, const int64_t* cid,
                     const double* coef, double* out);
void axpy(hipStream_t st, int64_t n, double a, const double* dx, double* x);
void lincomb(hipStream_t st, int64_t n, double a, const double* u, double b, const double* v, double* out);
void mul(hipStream_t st, int64_t n, const double* u, const double* v, double sgn, double* out);
// (zero != null: also zeroes zero[0, nzero) -- the scalar slots of the reduction that follows)
void dslacks_lin(hipStream_t st, int64_t n, int64_t m, const double* Cdx, bool has_lb, bool has_ub,
                 const double* dx, const double* dshp, double* ds, double* zero = nullptr, int nzero = 0);
// LP / QP / LP-phase-1 gradient pieces in one launch (k_lin_pieces)
struct LinPieces {
  int64_t n = 0, m = 0;
  const double *d = nullptr, *Cx = nullptr, *lb = nullptr, *ub = nullptr, *x = nullptr, *shp = nullptr;
  const double *c = nullptr, *Px = nullptr, *q = nullptr;
  double t = 0.0, add = 0.0;
  bool ph1 = false;
  double *s = nullptr, *inv = nullptr, *w = nullptr, *go = nullptr, *dvec = nullptr;
};
void lin_pieces(hipStream_t st, const LinPieces& a);
void slack_at(hipStream_t st, int64_t len, const double* s0, const double* ds, double a, double* out);
void reduce(hipStream_t st, const ReduceBatch& b, int count, double* out);

void cone_slacks(hipStream_t st, const SocpView& v, const double* Xx, const double* x, const double* lb,
                 const double* ub, const double* shp, double* lhs, double* rhs, double* s);
void cone_coef(hipStream_t st, int64_t K, const double* s, bool phase1, double* coef, double* invs);
void cone_rowweights(hipStream_t st, const SocpView& v, const double* coef, double* w);
void cone_grows(hipStream_t st, const SocpView& v, const double* lhs, const double* rhs, const double* coef);

int64_t ls_lin_blocks(int64_t len);
void ls_lin(hipStream_t st, int64_t len, int64_t bar_len, const double* s0, const double* ds, double alpha0,
            double beta, unsigned long long* pmask, double* psum);
void ls_cone(hipStream_t st, const SocpView& v, const double* lhs, const double* dlhs, const double* rhs,
             const double* drhs, const double* shp, const double* dshp, double alpha0, double beta,
             unsigned long long* pmask, double* psum);
void ls_fold(hipStream_t st, int64_t nblk, const unsigned long long* pmask, const double* psum,
             unsigned long long* mask_out, double* sum_out);
int64_t ls_resid_blocks(int64_t n, int64_t p);
void ls_resid(hipStream_t st, const ResidView& v, double alpha0, double beta, unsigned long long* pmask,
              double* psum);

void border(hipStream_t st, int64_t n, double* H, int64_t ldh, const double* hxs, const double* hssp);
void border_vec(hipStream_t st, int64_t n, const double* ct, const double* lbt, const double* ubt, double* out);
// the same from the inverse bound slacks (squared inside: one launch instead of three)
void border_vec_sq(hipStream_t st, int64_t n, const double* ct, const double* ilb, const double* iub, double* out);
void t_minus(hipStream_t st, double t, const double* sp, double* out);

}  // namespace ipm
