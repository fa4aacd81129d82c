// Native Newton engine + C ABI (include/ipm355.h).
//
// This file is the MI355X restatement of the reference's L1/L2 layers:
//   * the barrier oracle protocol of FunctionManager.py:94-195 (update_x / objective /
//     newton_objective / gradient / hessian, with the stale-slack semantics of Q2), and
//   * the Newton inner loops NewtonSolver.solve (NewtonSolver.py:80-206) and
//     NewtonSolverInfeasibleStart.solve (NewtonSolverInfeasibleStart.py:72-273), including the
//     Cholesky linear solves (NewtonSolver.py:277-341; NewtonSolverInfeasibleStart.py:386-538,
//     757-809) and their permanent LU fallback after a Cholesky failure (Q9).
// All vectors live on the device; each Newton iteration issues a fixed kernel sequence on one
// stream and performs ONE device->host copy (feasible start): the Cholesky info word, the
// 64-candidate feasibility mask, the 64 candidate barrier sums and ~12 scalars.  The
// backtracking decisions (incl. the reference's one-step Armijo lag, Q3) are then replayed
// exactly on the host from that table.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ipm355.h"
#include "ipm_barrier.h"
#include "ipm_common.h"
#include "ipm_handle.h"

using namespace ipm;

namespace {
constexpr double STEP_FLOOR = 1e-13;  // NewtonSolver.py:176, 190
constexpr int NCAND = 64;
// readback block layout (bytes): info (8 ints), mask (4 words), sums (NCAND), scal (64)
constexpr int RB_MASK = 32, RB_SUMS = 64, RB_SCAL = RB_SUMS + NCAND * 8;
constexpr int RB_INFO_TRSV_ERR = 4;   // info word 4: sticky device error word of the backward solve
constexpr int RB_INFO_LSQ = 5;        // info word 5: non-convergence of the least-squares eigensolver
constexpr int HOST_WORDS = IPM_HOST_WORDS;

enum Slot {
  SC_F0A = 0,  // c.x | x.Px | s
  SC_F0B,      // q.x
  SC_DFA,      // c.dx | x.Pdx | ds
  SC_DFB,      // q.dx
  SC_DDF,      // dx.Pdx
  SC_GX,       // g.x
  SC_GDX,      // g.dx
  SC_SUMLOG0,  // sum log(s0 + eps) over the barrier segment
  SC_SUMINV,   // phase 1: sum inv
  SC_SUMINV2,  // phase 1: sum inv^2
  SC_R0A,      // ||g + A^T v||^2
  SC_R0B,      // ||Ax - b||^2
  SC_XN,       // x[n]   (phase 1)
  SC_DXN,      // dx[n]  (phase 1)
  SC_COUNT
};
}  // namespace

struct ipm_problem {
  ipm_handle* h = nullptr;
  ipm_problem_desc d{};
  // dims / flags
  int64_t n = 0, N = 0, S = 0, Sbar = 0, nub = 0, nlb = 0, m = 0, p = 0, K = 0, R = 0, XR = 0, Lh = 0;
  int64_t ldh = 0, nbb = 0;  // ld of H, bound-segment length (SOCP)
  bool lp = false, qp = false, socp = false, ph1 = false, eq = false, diag = false, lu = false, lsq = false;
  SocpView sv{};
  // workspace carve
  double *xe = nullptr, *s0 = nullptr, *ds = nullptr, *inv = nullptr, *w = nullptr, *dvec = nullptr;
  double *g = nullptr, *go = nullptr, *gb = nullptr, *ct = nullptr, *Px = nullptr, *Pdx = nullptr;
  double *Cx = nullptr, *Cdx = nullptr, *dx = nullptr, *H = nullptr, *W2 = nullptr, *hxs = nullptr;
  double *scal = nullptr, *lhs0 = nullptr, *rhs0 = nullptr, *dlhs = nullptr, *drhs = nullptr;
  double *coef = nullptr, *ones = nullptr, *psum = nullptr, *sums = nullptr, *xd = nullptr;
  double *Ybuf = nullptr, *Sbuf = nullptr, *Wp = nullptr, *ATv = nullptr, *ATdv = nullptr, *Axb = nullptr;
  double *Adx = nullptr, *wv = nullptr, *r2 = nullptr, *tmpn = nullptr, *part = nullptr, *hdiag = nullptr;
  double *sdv = nullptr, *lhsd = nullptr, *rhsd = nullptr, *dv = nullptr, *tmpp = nullptr;
  unsigned long long *pmask = nullptr, *mask = nullptr;
  int64_t *piv = nullptr, *pivp = nullptr;
  int* info = nullptr;
  unsigned* ctl = nullptr;  // persistent-solve control words
  double* pws = nullptr;    // Cholesky panel workspace (inverted diagonal blocks)
  double* xinv = nullptr;   // backward solve: inverted 128 x 128 diagonal blocks of L
  int64_t part_elems = 0, nls_blocks = 0;
  std::vector<int64_t> rowcone_h, dslot_h;
  int64_t *rowcone_d = nullptr, *dslot_d = nullptr;
  bool use_backup = false;
  bool pieces_valid = false;  // barrier pieces (inv/coef/G) match the current slack state
  // w = inv^2 and dvec (with hess_add) were formed with the gradient (gradient_at's fused LP-family
  // path): assemble_hessian skips them while the slack state is unchanged
  bool hess_pre = false;
  double hess_add = 0.0;
  double* sws = nullptr;   // KKT SYRK split tail (syrk_split_ws_doubles)
  double* lsw = nullptr;   // least-squares workspace (lstsq_ws_doubles; null when the method never uses it)
};

// ------------------------------------------------------------------------- workspace
namespace {
struct Carver {
  char* base;
  int64_t off = 0;
  template <class T>
  T* take(int64_t count) {
    off = (off + 255) & ~int64_t(255);
    T* p = base ? reinterpret_cast<T*>(base + off) : nullptr;
    off += std::max<int64_t>(count, 1) * (int64_t)sizeof(T);
    return p;
  }
};

void derive(ipm_problem* pr) {
  const ipm_problem_desc& d = pr->d;
  pr->n = d.n;
  pr->ph1 = d.phase1 != 0;
  pr->N = d.n + (pr->ph1 ? 1 : 0);
  pr->lp = d.kind == IPM_KIND_LP;
  pr->qp = d.kind == IPM_KIND_QP;
  pr->socp = d.kind == IPM_KIND_SOCP;
  pr->m = d.C ? d.m : 0;
  pr->nub = d.ub ? d.n : 0;
  pr->nlb = d.lb ? d.n : 0;
  pr->p = d.A ? d.p : 0;
  pr->eq = pr->p > 0;
  pr->diag = d.solve_method == IPM_SOLVE_DIAGONAL || d.solve_method == IPM_SOLVE_DIAGONAL_LSTSQ;
  pr->lu = d.solve_method == IPM_SOLVE_LU;
  pr->lsq = d.solve_method == IPM_SOLVE_LSTSQ || d.solve_method == IPM_SOLVE_DIAGONAL_LSTSQ;
  if (pr->socp) {
    pr->K = d.K;
    pr->R = d.R;
    pr->XR = d.R + 2 * d.K;
    pr->nbb = pr->nub + pr->nlb;
    pr->S = pr->K + pr->nbb + pr->K;
    pr->Sbar = pr->K + pr->nbb;
    pr->Lh = d.R + d.Kd * d.n;
  } else {
    pr->S = pr->m + pr->nub + pr->nlb;
    pr->Sbar = pr->S;
  }
  // room for one bordered row (N+1 rows): the Newton right-hand side rides through the Cholesky
  // ... and a leading dimension of whole 128-byte lines: every 16-row block of a column of H is then
  // one cache line, so no line holds rows of two Cholesky roles (a line shared by a role that
  // stores and one that reads rows handed off inside the same launch could be served stale from an
  // XCD's L2: r6 saw 4 of 12 runs of the bordered n = 8193 trajectory differ with ld = 8194).
  // IPM_LDH_ALIGN (doubles; 2 = the round-5 layout) is a test knob, read per problem.
  const char* ela = getenv("IPM_LDH_ALIGN");
  const int64_t la = ela && atol(ela) >= 1 ? (int64_t)atol(ela) : 16;
  pr->ldh = (pr->N + 1 + la - 1) / la * la;
}

// leading dimension of the p x p Schur complement: whole 128-byte lines (as H's, derive())
static inline int64_t schur_ld(int64_t p) { return (p + 15) / 16 * 16; }

// the Newton step's Cholesky (potrf_lower_fused on the problem's stream)
static int potrf_step(ipm_problem* pr, hipStream_t st, int64_t n, double* H, int64_t ldh, int* info, double* ws,
                      int64_t ncols, const BorderJob* border = nullptr) {
  (void)pr;
  potrf_lower_fused(st, n, H, ldh, info, ws, ncols, border);
  return IPM_OK;
}

int64_t carve(ipm_problem* pr, char* base) {
  Carver c{base};
  const int64_t n = pr->n, N = pr->N, S = std::max<int64_t>(pr->S, 1), p = pr->p;
  pr->xe = c.take<double>(N);
  pr->xd = c.take<double>(N);
  pr->s0 = c.take<double>(S);
  pr->sdv = c.take<double>(S);
  pr->ds = c.take<double>(S);
  pr->inv = c.take<double>(S);
  pr->w = c.take<double>(std::max<int64_t>(pr->m, pr->XR) + 1);
  pr->dvec = c.take<double>(N);
  pr->hdiag = c.take<double>(N);
  pr->g = c.take<double>(N);
  pr->go = c.take<double>(N);
  pr->gb = c.take<double>(N);
  pr->ct = c.take<double>(N);
  pr->Px = c.take<double>(n);
  pr->Pdx = c.take<double>(n);
  pr->Cx = c.take<double>(std::max<int64_t>(pr->m, pr->XR) + 1);
  pr->Cdx = c.take<double>(std::max<int64_t>(pr->m, pr->XR) + 1);
  pr->dx = c.take<double>(N);
  pr->dv = c.take<double>(p + 1);
  pr->tmpn = c.take<double>(N);
  pr->tmpp = c.take<double>(p + 1);
  pr->hxs = c.take<double>(N);
  // the per-iteration readback block, contiguous (ONE device->host copy): info | mask | sums | scal
  {
    char* rb = c.take<char>(RB_SCAL + 64 * 8);
    pr->info = reinterpret_cast<int*>(rb);
    pr->mask = reinterpret_cast<unsigned long long*>(rb ? rb + RB_MASK : nullptr);
    pr->sums = reinterpret_cast<double*>(rb ? rb + RB_SUMS : nullptr);
    pr->scal = reinterpret_cast<double*>(rb ? rb + RB_SCAL : nullptr);
  }
  pr->ctl = c.take<unsigned>(8);
  pr->pws = c.take<double>(potrf_ws_doubles(std::max<int64_t>(N + 1, p)));
  pr->coef = c.take<double>(pr->K + 1);
  pr->ones = c.take<double>(pr->K + 1);
  pr->lhs0 = c.take<double>(pr->Lh + 1);
  pr->rhs0 = c.take<double>(pr->K + 1);
  pr->dlhs = c.take<double>(pr->Lh + 1);
  pr->drhs = c.take<double>(pr->K + 1);
  pr->lhsd = c.take<double>(pr->Lh + 1);
  pr->rhsd = c.take<double>(pr->K + 1);
  const int64_t nls = std::max<int64_t>(
      {ls_lin_blocks(pr->S), (pr->socp ? pr->K + ls_lin_blocks(pr->nbb) : 0), ls_resid_blocks(N, p)});
  pr->nls_blocks = nls;
  pr->pmask = c.take<unsigned long long>(nls + 1);
  pr->psum = c.take<double>((nls + 1) * NCAND);
  pr->H = c.take<double>(pr->ldh * (N + 1));
  pr->xinv = c.take<double>(trsv_inv_ws_doubles(N));
  pr->W2 = c.take<double>(N * std::max<int64_t>(p, 1));
  pr->piv = c.take<int64_t>(N);
  if (pr->eq) {
    pr->Ybuf = c.take<double>(N * p);
    pr->Sbuf = c.take<double>(schur_ld(p) * p);
    pr->Wp = c.take<double>(p);
    pr->ATv = c.take<double>(N);
    pr->ATdv = c.take<double>(N);
    pr->Axb = c.take<double>(p);
    pr->Adx = c.take<double>(p);
    pr->wv = c.take<double>(p);
    pr->r2 = c.take<double>(p);
    pr->pivp = c.take<int64_t>(p);
  }
  int64_t pe = gemv_t_ws_elems(std::max<int64_t>(pr->m, 1), std::max<int64_t>(n, 1));
  if (pr->socp) pe = std::max(pe, gemv_t_ws_elems(std::max<int64_t>(pr->XR, 1), n));
  if (pr->eq) pe = std::max(pe, gemv_t_ws_elems(p, n));
  pr->part_elems = pe;
  pr->part = c.take<double>(pe);
  if (!pr->diag && (pr->m > 0 || pr->socp)) pr->sws = c.take<double>(syrk_split_ws_doubles(n));
  // least squares (np_lstsq, and the Cholesky-failure backup Q9 of the feasible-start path): the
  // eigensolver's V (n^2) and scratch live in the problem workspace, never grown on the hot path
  {
    int64_t lw = 0;
    if (!pr->lu && !pr->diag && !pr->eq) lw = lstsq_ws_doubles(N, 1);
    if (pr->lsq && pr->eq && !pr->diag) lw = lstsq_ws_doubles(n, p) + lstsq_ws_doubles(p, 1) + p * schur_ld(p);
    if (pr->lsq && pr->diag && pr->eq) lw = lstsq_ws_doubles(p, 1);
    pr->lsw = lw > 0 ? c.take<double>(lw) : nullptr;
  }
  pr->rowcone_d = c.take<int64_t>(pr->R + 1);
  pr->dslot_d = c.take<int64_t>(pr->K + 1);
  return c.off + 256;
}

inline hipStream_t S(ipm_problem* pr) { return pr->h->stream; }

inline unsigned* trsv_err(ipm_problem* pr) { return reinterpret_cast<unsigned*>(pr->info + RB_INFO_TRSV_ERR); }
// the Jacobi eigensolver's info (lstsq_sym_factor) goes to its own word: the Cholesky info words
// keep meaning "factorization failed" (Q9), and a non-converged eigensolve surfaces at the readback
inline int* lsq_info(ipm_problem* pr) { return pr->info + RB_INFO_LSQ; }

// --------------------------------------------------------------- oracle pieces (L1)
// slack state (s, lhs, rhs) at point xp   (FunctionManager.py:118-149, 427-449, 933-994, 1258-1262)
void compute_slacks(ipm_problem* pr, const double* xp, double* s, double* lhs, double* rhs) {
  const ipm_problem_desc& d = pr->d;
  const double* shp = pr->ph1 ? xp + pr->n : nullptr;
  if (!pr->socp) {
    if (pr->m > 0) gemv_n(S(pr), pr->m, pr->n, 1.0, d.C, d.ldc, xp, 0.0, pr->Cx);
    slacks_lin(S(pr), pr->n, pr->m, d.d, pr->Cx, d.lb, d.ub, xp, shp, s);
  } else {
    gemv_n(S(pr), pr->R + pr->K, pr->n, 1.0, d.X, d.ldx, xp, 0.0, pr->Cx);
    cone_slacks(S(pr), pr->sv, pr->Cx, xp, d.lb, d.ub, shp, lhs, rhs, s);
  }
  pr->pieces_valid = false;
  pr->hess_pre = false;
}

// f(xp) pieces into scal slots (f0a, f0b): LP c.x ; QP/SOCP x.Px, q.x ; phase 1: s = xp[n].
// Requires Px = P xp computed (QP/SOCP with P).
void objective_parts(ipm_problem* pr, const double* xp, ReduceBatch& rb, int& cnt) {
  const ipm_problem_desc& d = pr->d;
  auto add = [&](const double* a, const double* b, int64_t len, int kind, int slot) {
    rb.ops[cnt++] = ReduceOp{a, b, len, 1, 1, kind, slot};
  };
  if (pr->ph1) {
    add(xp + pr->n, nullptr, 1, RED_SUM, SC_F0A);
    return;
  }
  if (pr->lp) {
    add(d.c, xp, pr->n, RED_DOT, SC_F0A);
  } else {
    if (d.P) add(xp, pr->Px, pr->n, RED_DOT, SC_F0A);
    if (d.q) add(d.q, xp, pr->n, RED_DOT, SC_F0B);
  }
}

// barrier pieces at slack state (s, lhs, rhs): inv / coef / G rows / ct, and the
// bound reciprocals.  t only enters the phase-1 s-component.
void barrier_pieces(ipm_problem* pr, const double* s, const double* lhs, const double* rhs) {
  const ipm_problem_desc& d = pr->d;
  hipStream_t st = S(pr);
  if (!pr->socp) {
    inv_eps(st, pr->S, s, 1e-15, pr->inv);
    if (pr->m > 0)
      gemv_t(st, pr->m, pr->n, 1.0, d.C, d.ldc, pr->inv, nullptr, 0.0, pr->ct, pr->part, pr->part_elems);
  } else {
    if (pr->ph1) {
      inv_eps(st, pr->Sbar, s, 1e-15, pr->inv);  // inv over the barrier segment
      cone_coef(st, pr->K, s, true, pr->coef, pr->inv);
    } else {
      cone_coef(st, pr->K, s, false, pr->coef, nullptr);
      // SOCP bound gradient terms use 1e-15 (FunctionManager.py:1093-1098)
      if (pr->nbb > 0) inv_eps(st, pr->nbb, s + pr->K, 1e-15, pr->inv + pr->K);
    }
    cone_grows(st, pr->sv, lhs, rhs, pr->coef);
    gemv_t(st, pr->K, pr->n, 1.0, d.X + (pr->R + pr->K) * d.ldx, d.ldx, pr->ones, nullptr, 0.0, pr->ct,
           pr->part, pr->part_elems);
  }
  pr->pieces_valid = true;
}

const double* inv_lb(ipm_problem* pr) {
  if (!pr->d.lb) return nullptr;
  return pr->socp ? pr->inv + pr->K + pr->nub : pr->inv + pr->m + pr->nub;
}
const double* inv_ub(ipm_problem* pr) {
  if (!pr->d.ub) return nullptr;
  return pr->socp ? pr->inv + pr->K : pr->inv + pr->m;
}
const double* s_lb(ipm_problem* pr, const double* s) {
  if (!pr->d.lb) return nullptr;
  return pr->socp ? s + pr->K + pr->nub : s + pr->m + pr->nub;
}
const double* s_ub(ipm_problem* pr, const double* s) {
  if (!pr->d.ub) return nullptr;
  return pr->socp ? s + pr->K : s + pr->m;
}

// objective gradient at xp: go = t c | (P xp + q) t ; also leaves Px
void objective_grad(ipm_problem* pr, const double* xp, double t) {
  const ipm_problem_desc& d = pr->d;
  if (pr->ph1) return;
  if (pr->lp) {
    objgrad(S(pr), pr->n, t, d.c, nullptr, nullptr, pr->go);
  } else {
    if (d.P) gemv_n(S(pr), pr->n, pr->n, 1.0, d.P, d.ldp, xp, 0.0, pr->Px);
    objgrad(S(pr), pr->n, t, nullptr, d.P ? pr->Px : nullptr, d.q, pr->go);
  }
}

// full gradient at xp with slack state (s, ...) whose pieces are computed: g = go + barrier
// (FunctionManager.py:232-265, 509-545, 741-781, 1055-1102, 1322-1370)
void assemble_gradient(ipm_problem* pr, double t, const double* s, double* g) {
  hipStream_t st = S(pr);
  const double* go = pr->ph1 ? nullptr : pr->go;
  const bool ctf = pr->socp || pr->ph1;
  const double* ct = (pr->m > 0 || pr->socp) ? pr->ct : nullptr;
  grad_combine(st, pr->n, go, inv_lb(pr), inv_ub(pr), ct, ctf, g);
  if (pr->ph1) {
    ReduceBatch rb{};
    rb.ops[0] = ReduceOp{pr->inv, nullptr, pr->Sbar, 1, 1, RED_SUM, SC_SUMINV};
    reduce(st, rb, 1, pr->scal);
    t_minus(st, t, pr->scal + SC_SUMINV, g + pr->n);
  }
  (void)s;
}

// barrier-only gradient B (used by the infeasible-start residual with stale slacks):
// B = -blb + bub + ct  (go added inside the residual kernel)
void assemble_barrier_grad(ipm_problem* pr, double* B) {
  const bool ctf = pr->socp;
  const double* ct = (pr->m > 0 || pr->socp) ? pr->ct : nullptr;
  grad_combine(S(pr), pr->n, nullptr, inv_lb(pr), inv_ub(pr), ct, ctf, B);
}

// Hessian into H (column-major lower, ldh) -- or the diagonal vector hdiag for the
// diagonal strategy.  Requires barrier_pieces at the same slack state.
// (FunctionManager.py:267-326, 547-611, 783-827, 1104-1158, 1372-1453)
void assemble_hessian(ipm_problem* pr, double t, const double* s, bool psd) {
  const ipm_problem_desc& d = pr->d;
  hipStream_t st = S(pr);
  const double add = psd ? 1e-9 : 0.0;
  ipm_handle* h = pr->h;
  if (h->timing) { hipEventRecord(h->ev[0], st); h->kkt_pending = true; }
  if (pr->diag) {
    // diag vector WITH eps: inv_lb^2 (+ inv_ub^2)   (FunctionManager.py:283-292)
    dvec_sq(st, pr->n, inv_lb(pr), inv_ub(pr), 0.0, pr->hdiag);
    if (h->timing) hipEventRecord(h->ev[1], st);
    return;
  }
  SyrkEpi e;
  if (!pr->socp) {
    const bool pre = pr->hess_pre && pr->hess_add == add && s == pr->s0;
    if (pr->m > 0 && !pre) square(st, pr->m, pr->inv, pr->w);
    if (pr->ph1) {
      if (!pre) dvec_sq(st, pr->n, inv_lb(pr), inv_ub(pr), add, pr->dvec);
    } else {
      if (!pre) dvec_inv_sq(st, pr->n, s_lb(pr, s), s_ub(pr, s), add, pr->dvec);
      if (pr->qp) { e.P = d.P; e.ldp = d.ldp; e.tP = t; }
    }
    e.dvec = pr->dvec;
    if (pr->sws) { e.split_ws = pr->sws; e.split_cap = syrk_split_cap(pr->n); e.flags_zero = true; }
    syrk_lower(st, pr->n, pr->m, 1.0, d.C, d.ldc, nullptr, 0, pr->w, 0.0, pr->H, pr->ldh, e);
    if (pr->ph1) {
      // border: hxs = -C^T inv_C^2 + inv_lb^2 - inv_ub^2 ; hss = sum inv^2 (+psd)
      if (pr->m > 0)
        gemv_t(st, pr->m, pr->n, 1.0, d.C, d.ldc, pr->inv, pr->inv, 0.0, pr->ct, pr->part, pr->part_elems);
      border_vec_sq(st, pr->n, pr->m > 0 ? pr->ct : nullptr, d.lb ? inv_lb(pr) : nullptr, d.ub ? inv_ub(pr) : nullptr,
                    pr->hxs);
      ReduceBatch rb{};
      rb.ops[0] = ReduceOp{pr->inv, nullptr, pr->S, 1, 1, RED_SUMSQ, SC_SUMINV2};
      reduce(st, rb, 1, pr->scal);
      border(st, pr->n, pr->H, pr->ldh, pr->hxs, pr->scal + SC_SUMINV2);
    }
  } else {
    cone_rowweights(st, pr->sv, pr->coef, pr->w);
    if (pr->ph1) dvec_sq(st, pr->n, inv_lb(pr), inv_ub(pr), add, pr->dvec);
    else dvec_inv_eps_sq(st, pr->n, s_lb(pr, s), s_ub(pr, s), add, pr->dvec);
    if (d.Kd > 0) dvec_diag_cones(st, pr->n, d.Kd, d.Ad, d.dcone_id, pr->coef, pr->dvec);
    if (d.P && !pr->ph1) { e.P = d.P; e.ldp = d.ldp; e.tP = t; }
    e.dvec = pr->dvec;
    if (pr->sws) { e.split_ws = pr->sws; e.split_cap = syrk_split_cap(pr->n); e.flags_zero = true; }
    syrk_lower(st, pr->n, pr->XR, 1.0, d.X, d.ldx, nullptr, 0, pr->w, 0.0, pr->H, pr->ldh, e);
    if (pr->ph1) {
      // hxs = -sum_i G_i inv_i + inv_lb^2 - inv_ub^2 ; hss = sum inv^2 (barrier segment)
      gemv_t(st, pr->K, pr->n, 1.0, d.X + (pr->R + pr->K) * d.ldx, d.ldx, pr->inv, nullptr, 0.0, pr->ct,
             pr->part, pr->part_elems);
      border_vec_sq(st, pr->n, pr->ct, d.lb ? inv_lb(pr) : nullptr, d.ub ? inv_ub(pr) : nullptr, pr->hxs);
      ReduceBatch rb{};
      rb.ops[0] = ReduceOp{pr->inv, nullptr, pr->Sbar, 1, 1, RED_SUMSQ, SC_SUMINV2};
      reduce(st, rb, 1, pr->scal);
      border(st, pr->n, pr->H, pr->ldh, pr->hxs, pr->scal + SC_SUMINV2);
    }
  }
  pr->hess_pre = false;   // (the Cholesky overwrites nothing of w / dvec, but a fallback may rebuild H with another add)
  if (pr->ph1 && psd) {
    // corner += 1e-9 (NewtonSolver.py:269-275 adds 1e-9 to the whole (n+1) diagonal); ones[0] == 1
    axpy(st, 1, 1e-9, pr->ones, pr->H + pr->n * pr->ldh + pr->n);
  }
  if (h->timing) hipEventRecord(h->ev[1], st);
}

void host_sync_copy(ipm_problem* pr, const void* dsrc, size_t bytes, void* hdst) {
  hipMemcpyAsync(hdst, dsrc, bytes, hipMemcpyDeviceToHost, S(pr));
  hipStreamSynchronize(S(pr));
}

}  // namespace

// ======================================================================= C ABI: handle
extern "C" int ipm_version(void) { return 1; }

extern "C" int ipm_create(int device, void* stream, ipm_handle** out) {
  if (!out) return IPM_INVALID_ARG;
  ipm_handle* h = new ipm_handle();
  h->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) { delete h; return IPM_HIP_ERROR; }
  // NULL = the legacy default stream (what torch's default stream is), so work is ordered
  // with the caller's tensor initialisation and reads without extra events.
  h->stream = (hipStream_t)stream;
  if (hipHostMalloc((void**)&h->hbuf, HOST_WORDS * sizeof(double)) != hipSuccess) { delete h; return IPM_HIP_ERROR; }
  if (hipMalloc((void**)&h->dinfo, 64) != hipSuccess) { delete h; return IPM_HIP_ERROR; }
  h->ctl = reinterpret_cast<unsigned*>(h->dinfo + 8);
  for (auto& ev : h->ev) hipEventCreate(&ev);
  *out = h;
  return IPM_OK;
}

extern "C" int ipm_destroy(ipm_handle* h) {
  if (!h) return IPM_OK;
  hipStreamSynchronize(h->stream);
  if (h->hbuf) hipHostFree(h->hbuf);
  if (h->dinfo) hipFree(h->dinfo);
  if (h->pws) hipFree(h->pws);
  if (h->scratch) hipFree(h->scratch);
  lstsq_release(h->rb);
  for (auto& ev : h->ev) hipEventDestroy(ev);
  if (h->own_stream) hipStreamDestroy(h->stream);
  delete h;
  return IPM_OK;
}

extern "C" const char* ipm_last_error(ipm_handle* h) { return h ? h->err.c_str() : "null handle"; }

static double* scratch(ipm_handle* h, size_t bytes) { return ipm_handle_scratch(h, bytes); }

// ======================================================================= level 0
extern "C" int ipm_gemv(ipm_handle* h, int trans, int64_t rows, int64_t cols, double alpha, const double* M,
                        int64_t ldm, const double* x, double beta, double* y) {
  if (!h || rows < 0 || cols < 0 || ldm < cols) return IPM_INVALID_ARG;
  if (!trans) {
    gemv_n(h->stream, rows, cols, alpha, M, ldm, x, beta, y);
  } else {
    const int64_t pe = gemv_t_ws_elems(std::max<int64_t>(rows, 1), std::max<int64_t>(cols, 1));
    double* part = scratch(h, pe * sizeof(double));
    if (!part) return IPM_HIP_ERROR;
    gemv_t(h->stream, rows, cols, alpha, M, ldm, x, nullptr, beta, y, part, pe);
  }
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_syrk(ipm_handle* h, int64_t n, int64_t k, const double* X, int64_t ldx, const double* w,
                        double alpha, double beta, double* H, int64_t ldh) {
  if (!h || n < 0 || k < 0 || ldh < n || (k > 0 && ldx < n)) return IPM_INVALID_ARG;
  SyrkEpi e;
  // the KKT SYRK's split tail (handle scratch), as inside the Newton step
  if (double* sw = scratch(h, (size_t)syrk_split_ws_doubles(n) * sizeof(double))) {
    e.split_ws = sw;
    e.split_cap = syrk_split_cap(n);
  }
  syrk_lower(h->stream, n, k, alpha, X, ldx, nullptr, 0, w, beta, H, ldh, e);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_potrf(ipm_handle* h, int64_t n, double* H, int64_t ldh, int* info) {
  return ipm_potrf_partial(h, n, n, H, ldh, info);
}

extern "C" int ipm_potrf_partial(ipm_handle* h, int64_t n, int64_t ncols, double* H, int64_t ldh, int* info) {
  if (!h || n < 0 || ldh < n || ncols < 0 || ncols > n) return IPM_INVALID_ARG;
  if (n > h->pws_n) {
    if (h->pws) hipFree(h->pws);
    h->pws = nullptr;
    h->pws_n = 0;
    HIPCHK(h, hipMalloc((void**)&h->pws, potrf_ws_doubles(n) * sizeof(double)));
    h->pws_n = n;
  }
  // the fused factorization hands rows between workgroups inside each launch; it is run on a
  // matrix whose columns start on 128-byte lines (no line holds rows of two roles: the solver's
  // own matrices are laid out that way).  Any other layout is factored in an aligned copy.
  if ((ldh % 16) != 0 || (reinterpret_cast<uintptr_t>(H) & 127) != 0) {
    const int64_t ld2 = (n + 15) / 16 * 16;
    double* tmp = nullptr;
    if (n > 0) {
      HIPCHK(h, hipMallocAsync((void**)&tmp, (size_t)(ld2 * n) * sizeof(double), h->stream));
      HIPCHK(h, hipMemcpy2DAsync(tmp, ld2 * sizeof(double), H, ldh * sizeof(double), n * sizeof(double), n,
                                 hipMemcpyDeviceToDevice, h->stream));
    }
    potrf_lower_fused(h->stream, n, tmp, ld2, h->dinfo, h->pws, ncols);
    if (n > 0) {
      HIPCHK(h, hipMemcpy2DAsync(H, ldh * sizeof(double), tmp, ld2 * sizeof(double), n * sizeof(double), ncols,
                                 hipMemcpyDeviceToDevice, h->stream));
      HIPCHK(h, hipFreeAsync(tmp, h->stream));
    }
  } else {
    potrf_lower_fused(h->stream, n, H, ldh, h->dinfo, h->pws, ncols);
  }
  HIPCHK(h, hipMemcpyAsync(h->hbuf, h->dinfo, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  int inf;
  std::memcpy(&inf, h->hbuf, sizeof(int));
  if (info) *info = inf;
  if (inf < 0) {
    h->err = "Cholesky: a wait inside the factorization ran past its wall-clock bound (info " + std::to_string(inf) +
             "); the factor is not valid";
    return IPM_HIP_ERROR;
  }
  return inf == 0 ? IPM_OK : IPM_NOT_POSITIVE_DEFINITE;
}

extern "C" int ipm_potrs(ipm_handle* h, int64_t n, int64_t nrhs, const double* L, int64_t ldl, double* B,
                         int64_t ldb) {
  if (!h || n < 0 || nrhs < 0 || ldl < n || ldb < nrhs) return IPM_INVALID_ARG;
  if (nrhs >= 32 && n >= 128) {
    double* W = scratch(h, potrs_blocked_ws_doubles(n, nrhs) * sizeof(double));
    if (!W) return IPM_HIP_ERROR;
    potrs_blocked(h->stream, n, nrhs, L, ldl, B, ldb, W);
    HIPCHK(h, hipGetLastError());
    return IPM_OK;
  }
  const int64_t wn = (std::max<int64_t>(n * ldb, 1) + 31) & ~int64_t(31);
  double* W = scratch(h, (wn + trsv_inv_ws_doubles(n)) * sizeof(double));
  if (!W) return IPM_HIP_ERROR;
  unsigned* err = h->ctl + 7;   // potrs_lower uses ctl[0..3]
  HIPCHK(h, hipMemsetAsync(err, 0, sizeof(unsigned), h->stream));
  potrs_lower(h->stream, n, nrhs, L, ldl, B, ldb, W, h->ctl, W + wn, err);
  HIPCHK(h, hipGetLastError());
  if (nrhs == 1 && ldb == 1) {
    HIPCHK(h, hipMemcpyAsync(h->hbuf, err, sizeof(unsigned), hipMemcpyDeviceToHost, h->stream));
    HIPCHK(h, hipStreamSynchronize(h->stream));
    unsigned e;
    std::memcpy(&e, h->hbuf, sizeof(unsigned));
    if (e) {
      h->err = "backward solve: a chain producer did not publish within the spin bound";
      return IPM_HIP_ERROR;
    }
  }
  return IPM_OK;
}

extern "C" int ipm_getrf(ipm_handle* h, int64_t n, double* A, int64_t lda, int64_t* piv, int* info) {
  if (!h || n < 0 || lda < n || !piv) return IPM_INVALID_ARG;
  if (n == 0) return IPM_OK;
  double* lw = scratch(h, (size_t)getrf_ws_doubles(n) * sizeof(double));
  if (!lw) { h->err = "scratch alloc failed"; return IPM_HIP_ERROR; }
  getrf(h->stream, n, A, lda, piv, h->dinfo, lw);
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (info) *info = 0;
  return IPM_OK;
}

extern "C" int ipm_getrs(ipm_handle* h, int64_t n, int64_t nrhs, const double* LU, int64_t lda, const int64_t* piv,
                         double* B, int64_t ldb) {
  if (!h || n < 0 || nrhs < 0 || lda < n || ldb < nrhs) return IPM_INVALID_ARG;
  if (n > 0 && nrhs > 0) getrs(h->stream, n, nrhs, LU, lda, piv, B, ldb);
  HIPCHK(h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_lstsq_sym(ipm_handle* h, int64_t n, int64_t nrhs, double* A, int64_t lda, double* B, int64_t ldb,
                             int* info) {
  if (!h || n < 0 || nrhs < 0 || lda < n || ldb < nrhs) return IPM_INVALID_ARG;
  if (info) *info = 0;
  if (n == 0 || nrhs == 0) return IPM_OK;
  double* lw = scratch(h, (size_t)lstsq_ws_doubles(n, nrhs) * sizeof(double));
  if (!lw) { h->err = "scratch alloc failed"; return IPM_HIP_ERROR; }
  HIPCHK(h, hipMemsetAsync(h->dinfo, 0, sizeof(int), h->stream));   // (the factor's info is sticky)
  if (lstsq_sym_factor(&h->rb, h->stream, n, A, lda, lw, h->dinfo) ||
      lstsq_sym_apply(&h->rb, h->stream, n, nrhs, A, lda, B, ldb, lw)) {
    h->err = "least-squares library call failed";
    return IPM_HIP_ERROR;
  }
  HIPCHK(h, hipGetLastError());
  HIPCHK(h, hipMemcpyAsync(h->hbuf, h->dinfo, sizeof(int), hipMemcpyDeviceToHost, h->stream));
  HIPCHK(h, hipStreamSynchronize(h->stream));
  int inf;
  std::memcpy(&inf, h->hbuf, sizeof(int));
  if (info) *info = inf;
  return IPM_OK;
}

extern "C" int ipm_last_timings(ipm_handle* h, double* kkt_ms, double* potrf_ms, double* count) {
  // averages over the Newton iterations since ipm_set_timing(h, 1)
  if (!h) return IPM_INVALID_ARG;
  HIPCHK(h, hipStreamSynchronize(h->stream));
  if (kkt_ms) *kkt_ms = h->kkt_cnt ? h->kkt_sum / h->kkt_cnt : 0.0;
  if (potrf_ms) *potrf_ms = h->potrf_cnt ? h->potrf_sum / h->potrf_cnt : 0.0;
  if (count) *count = (double)h->kkt_cnt;
  return IPM_OK;
}

extern "C" int ipm_kkt_flops(ipm_problem* pr, double* upfront, double* deferred) {
  // KKT SYRK flops (SYRK convention: 2 per multiply-add over the lower triangle incl. diagonal);
  // all of it runs in the up-front SYRK kernel (deferred: 0, kept for ABI compatibility)
  if (!pr) return IPM_INVALID_ARG;
  const double n = (double)pr->n;
  const double m = (double)(pr->socp ? pr->XR : pr->m);
  if (upfront) *upfront = m * n * (n + 1);
  if (deferred) *deferred = 0.0;
  return IPM_OK;
}

// HIP-event time (ms, average over reps, on the handle's stream) of the HBM-bound kernels of one
// Newton step on this problem's own buffers: [0] the slack GEMV C x (k_gemv_n), [1] the gradient
// GEMV C^T w (k_gemv_t_part + its fold), [2] one 64-candidate line-search pass over the slacks
// (k_ls_lin).  Clobbers only scratch (Cx, part, pmask/psum).  LP/QP problems with C only.
extern "C" int ipm_time_hbm_kernels(ipm_problem* pr, int reps, double* ms) {
  if (!pr || reps <= 0 || !ms || pr->socp || pr->m <= 0) return IPM_INVALID_ARG;
  ipm_handle* h = pr->h;
  hipStream_t st = h->stream;
  const ipm_problem_desc& d = pr->d;
  hipEvent_t e0, e1;
  HIPCHK(h, hipEventCreate(&e0));
  HIPCHK(h, hipEventCreate(&e1));
  for (int k = 0; k < 3; ++k) {
    auto launch = [&]() {
      if (k == 0) gemv_n(st, pr->m, pr->n, 1.0, d.C, d.ldc, pr->xe, 0.0, pr->Cx);
      else if (k == 1) gemv_t(st, pr->m, pr->n, 1.0, d.C, d.ldc, pr->w, nullptr, 0.0, pr->tmpn, pr->part, pr->part_elems);
      else ls_lin(st, pr->S, pr->Sbar, pr->s0, pr->ds, 1.0, 0.5, pr->pmask, pr->psum);
    };
    launch();   // warm
    hipEventRecord(e0, st);
    for (int r = 0; r < reps; ++r) launch();
    hipEventRecord(e1, st);
    HIPCHK(h, hipEventSynchronize(e1));
    float t = 0.f;
    hipEventElapsedTime(&t, e0, e1);
    ms[k] = (double)t / reps;
  }
  hipEventDestroy(e0);
  hipEventDestroy(e1);
  return IPM_OK;
}

// sizes the HBM-kernel byte counts need: m, n, S (slacks incl. bounds)
extern "C" int ipm_problem_sizes(ipm_problem* pr, int64_t* out) {
  if (!pr || !out) return IPM_INVALID_ARG;
  out[0] = pr->m;
  out[1] = pr->n;
  out[2] = pr->S;
  return IPM_OK;
}

extern "C" int ipm_debug_set_trsv_spin_limit(unsigned limit) {
  set_trsv_spin_limit(limit);
  return IPM_OK;
}

extern "C" int ipm_debug_set_potrf_spin_limit(unsigned microseconds) {
  set_potrf_spin_limit_us(microseconds);
  return IPM_OK;
}

extern "C" int ipm_debug_lstsq_fail_call(int k) {
  set_lstsq_fail_call(k);
  return IPM_OK;
}

extern "C" int ipm_debug_set_trsv_publish_delay(int ticket) {
  set_trsv_publish_delay(ticket);
  return IPM_OK;
}

extern "C" int ipm_set_timing(ipm_handle* h, int on) {
  if (!h) return IPM_INVALID_ARG;
  h->timing = on != 0;
  h->kkt_sum = h->potrf_sum = 0.0;
  h->kkt_cnt = h->potrf_cnt = 0;
  h->kkt_pending = h->potrf_pending = false;
  return IPM_OK;
}

// ======================================================================= problems
extern "C" int64_t ipm_workspace_bytes(const ipm_problem_desc* desc) {
  if (!desc) return -1;
  ipm_problem tmp;
  tmp.d = *desc;
  derive(&tmp);
  return carve(&tmp, nullptr);
}

extern "C" int ipm_problem_create(ipm_handle* h, const ipm_problem_desc* desc, void* workspace,
                                  int64_t workspace_bytes, ipm_problem** out) {
  if (!h || !desc || !out) return IPM_INVALID_ARG;
  const ipm_problem_desc& d = *desc;
  if (d.n <= 0) { h->err = "n must be positive"; return IPM_INVALID_ARG; }
  if (d.kind == IPM_KIND_LP && !d.phase1 && !d.c) { h->err = "LP needs c"; return IPM_INVALID_ARG; }
  if (d.kind == IPM_KIND_QP && !d.P) { h->err = "QP needs P"; return IPM_INVALID_ARG; }
  if (d.C && (d.m <= 0 || !d.d || d.ldc < d.n)) { h->err = "bad C/d"; return IPM_INVALID_ARG; }
  if (d.A && (d.p <= 0 || !d.AT || !d.b || d.lda < d.n)) { h->err = "bad A/AT/b"; return IPM_INVALID_ARG; }
  if (d.kind == IPM_KIND_SOCP && (d.K <= 0 || !d.X || !d.cone_row_off_host)) {
    h->err = "SOCP needs cones";
    return IPM_INVALID_ARG;
  }
  if (d.phase1 && d.kind != IPM_KIND_SOCP && !d.C) { h->err = "LP phase 1 needs C"; return IPM_INVALID_ARG; }
  ipm_problem* pr = new ipm_problem();
  pr->h = h;
  pr->d = d;
  derive(pr);
  const int64_t need = carve(pr, nullptr);
  if (!workspace || workspace_bytes < need) {
    h->err = "workspace too small: need " + std::to_string(need);
    delete pr;
    return IPM_INVALID_ARG;
  }
  carve(pr, reinterpret_cast<char*>(workspace));
  hipMemsetAsync(pr->info, 0, RB_MASK, h->stream);   // info words incl. the sticky device error word
  if (pr->sws) {   // the KKT SYRK's split / stream-K flags: zeroed once, left zero by the kernels
    const int64_t cap = syrk_split_cap(pr->n);
    hipMemsetAsync(pr->sws + cap * 128 * 128, 0, (syrk_split_ws_doubles(pr->n) - cap * 128 * 128) * sizeof(double),
                   h->stream);
  }
  pr->use_backup = d.solve_method == IPM_SOLVE_LU || d.solve_method == IPM_SOLVE_LSTSQ;
  if (pr->socp) {
    // host-side structure: row -> cone, cone -> diagonal slot
    pr->rowcone_h.assign(pr->R + 1, 0);
    pr->dslot_h.assign(pr->K + 1, -1);
    for (int64_t i = 0; i < pr->K; ++i)
      for (int64_t r = d.cone_row_off_host[i]; r < d.cone_row_off_host[i + 1]; ++r) pr->rowcone_h[r] = i;
    for (int64_t c = 0; c < d.Kd; ++c) pr->dslot_h[d.dcone_id_host[c]] = c;
    hipMemcpyAsync(pr->rowcone_d, pr->rowcone_h.data(), (pr->R + 1) * sizeof(int64_t), hipMemcpyHostToDevice,
                   h->stream);
    hipMemcpyAsync(pr->dslot_d, pr->dslot_h.data(), (pr->K + 1) * sizeof(int64_t), hipMemcpyHostToDevice,
                   h->stream);
    fill(h->stream, pr->ones, pr->K + 1, 1.0);
    SocpView& v = pr->sv;
    v.n = pr->n; v.K = pr->K; v.R = pr->R; v.Kd = d.Kd; v.nbnd = pr->nbb;
    v.X = d.X; v.ldx = d.ldx; v.off = d.cone_row_off; v.rowcone = pr->rowcone_d; v.dslot = pr->dslot_d;
    v.cb = d.cone_b; v.cd = d.cone_d; v.has_c = d.has_cone_c; v.Ad = d.Ad; v.bd = d.bd;
    // zero the G rows (and c rows if absent) once
    hipMemsetAsync(d.X + (pr->R + pr->K) * d.ldx, 0, pr->K * d.ldx * sizeof(double), h->stream);
  } else {
    fill(h->stream, pr->ones, pr->K + 1, 1.0);
  }
  HIPCHK(h, hipStreamSynchronize(h->stream));
  *out = pr;
  return IPM_OK;
}

extern "C" int ipm_problem_destroy(ipm_problem* pr) {
  delete pr;
  return IPM_OK;
}

extern "C" int ipm_get_use_backup(ipm_problem* pr) { return pr && pr->use_backup ? 1 : 0; }
extern "C" int ipm_set_use_backup(ipm_problem* pr, int f) {
  if (!pr) return IPM_INVALID_ARG;
  pr->use_backup = f != 0;
  return IPM_OK;
}

// ======================================================================= oracle protocol
extern "C" int ipm_fm_update_x(ipm_problem* pr, const double* x, int update_slacks) {
  if (!pr || !x) return IPM_INVALID_ARG;
  copy(S(pr), pr->xe, x, pr->N);
  if (update_slacks) compute_slacks(pr, pr->xe, pr->s0, pr->lhs0, pr->rhs0);
  HIPCHK(pr->h, hipGetLastError());
  return IPM_OK;
}

extern "C" int64_t ipm_fm_num_slacks(ipm_problem* pr) { return pr ? pr->S : -1; }

extern "C" int ipm_fm_slacks(ipm_problem* pr, double* out) {
  if (!pr || !out) return IPM_INVALID_ARG;
  copy(S(pr), out, pr->s0, pr->S);
  HIPCHK(pr->h, hipGetLastError());
  return IPM_OK;
}

static int fm_objective_value(ipm_problem* pr, double* f) {
  ReduceBatch rb{};
  int cnt = 0;
  if (!pr->ph1 && !pr->lp && pr->d.P) gemv_n(S(pr), pr->n, pr->n, 1.0, pr->d.P, pr->d.ldp, pr->xe, 0.0, pr->Px);
  objective_parts(pr, pr->xe, rb, cnt);
  fill(S(pr), pr->scal, 2, 0.0);
  reduce(S(pr), rb, cnt, pr->scal);
  HIPCHK(pr->h, hipMemcpyAsync(pr->h->hbuf, pr->scal, 2 * sizeof(double), hipMemcpyDeviceToHost, S(pr)));
  HIPCHK(pr->h, hipStreamSynchronize(S(pr)));
  const double a = pr->h->hbuf[0], b = pr->h->hbuf[1];
  if (pr->ph1 || pr->lp) *f = a;
  else {
    double v = 0.0;
    if (pr->d.P) v = v + 1.0 / 2.0 * a;
    if (pr->d.q) v = v + b;
    *f = v;
  }
  return IPM_OK;
}

extern "C" int ipm_fm_objective(ipm_problem* pr, double* out) {
  if (!pr || !out) return IPM_INVALID_ARG;
  return fm_objective_value(pr, out);
}

extern "C" int ipm_fm_newton_objective(ipm_problem* pr, double t, double* out) {
  if (!pr || !out) return IPM_INVALID_ARG;
  double f;
  int rc = fm_objective_value(pr, &f);
  if (rc) return rc;
  double val = t * f;
  if (pr->Sbar > 0) {
    ReduceBatch rb{};
    rb.ops[0] = ReduceOp{pr->s0, nullptr, pr->Sbar, 1, 1, RED_SUMLOG, SC_SUMLOG0};
    reduce(S(pr), rb, 1, pr->scal);
    HIPCHK(pr->h, hipMemcpyAsync(pr->h->hbuf, pr->scal + SC_SUMLOG0, sizeof(double), hipMemcpyDeviceToHost, S(pr)));
    HIPCHK(pr->h, hipStreamSynchronize(S(pr)));
    val = val - pr->h->hbuf[0];
  }
  *out = val;
  return IPM_OK;
}

extern "C" int ipm_fm_gradient(ipm_problem* pr, double t, double* g) {
  if (!pr || !g) return IPM_INVALID_ARG;
  objective_grad(pr, pr->xe, t);
  barrier_pieces(pr, pr->s0, pr->lhs0, pr->rhs0);
  assemble_gradient(pr, t, pr->s0, g);
  HIPCHK(pr->h, hipGetLastError());
  return IPM_OK;
}

extern "C" int ipm_fm_hessian(ipm_problem* pr, double t, double* Hout, int64_t ldo) {
  if (!pr || !Hout) return IPM_INVALID_ARG;
  barrier_pieces(pr, pr->s0, pr->lhs0, pr->rhs0);
  assemble_hessian(pr, t, pr->s0, false);
  if (pr->diag) copy(S(pr), Hout, pr->hdiag, pr->n);
  else sym_lower_to_full(S(pr), pr->N, pr->H, pr->ldh, Hout, ldo);
  HIPCHK(pr->h, hipGetLastError());
  return IPM_OK;
}

// ======================================================================= Newton engine
namespace {

struct HostTable {
  std::vector<double> alpha;  // alpha_k = beta^k by repeated multiplication (host == device bits)
  void build(double beta, int64_t upto) {
    if ((int64_t)alpha.size() > upto) return;
    if (alpha.empty()) alpha.push_back(1.0);
    while ((int64_t)alpha.size() <= upto) alpha.push_back(alpha.back() * beta);
  }
};

// zero_scal: the slack-direction launch also zeroes the scalar slots (enqueue_scalars(.., true)
// then skips its fill); C dx and P dx share one GEMV launch (LP family)
void prep_linesearch_dirs(ipm_problem* pr, bool zero_scal = false) {
  const ipm_problem_desc& d = pr->d;
  hipStream_t st = S(pr);
  const double* dsh = pr->ph1 ? pr->dx + pr->n : nullptr;
  if (!pr->socp) {
    const bool qpP = !pr->lp && !pr->ph1 && d.P;
    if (pr->m > 0 && qpP) gemv_n2(st, pr->n, pr->dx, pr->m, d.C, d.ldc, pr->Cdx, pr->n, d.P, d.ldp, pr->Pdx);
    else if (pr->m > 0) gemv_n(st, pr->m, pr->n, 1.0, d.C, d.ldc, pr->dx, 0.0, pr->Cdx);
    dslacks_lin(st, pr->n, pr->m, pr->Cdx, d.lb != nullptr, d.ub != nullptr, pr->dx, dsh, pr->ds,
                zero_scal ? pr->scal : nullptr, SC_COUNT);
    if (qpP && pr->m <= 0) gemv_n(st, pr->n, pr->n, 1.0, d.P, d.ldp, pr->dx, 0.0, pr->Pdx);
    return;
  } else {
    // dlhs: dense rows from X dx; diagonal cones a * dx ; drhs = c_i.dx (0 without c).  The X dx
    // rows go straight to dlhs and drhs (one launch; round 5 formed X dx in Cdx and copied both
    // parts out: two device copies per Newton step, r6 trace)
    if (d.has_cone_c) {
      gemv_n2(st, pr->n, pr->dx, pr->R, d.X, d.ldx, pr->dlhs, pr->K, d.X + pr->R * d.ldx, d.ldx, pr->drhs);
    } else {
      gemv_n(st, pr->R, pr->n, 1.0, d.X, d.ldx, pr->dx, 0.0, pr->dlhs);
      fill(st, pr->drhs, pr->K, 0.0);
    }
    for (int64_t c = 0; c < d.Kd; ++c) mul(st, pr->n, d.Ad + c * pr->n, pr->dx, 1.0, pr->dlhs + pr->R + c * pr->n);
    if (pr->nbb > 0) dslacks_lin(st, pr->n, 0, nullptr, d.lb != nullptr, d.ub != nullptr, pr->dx, dsh, pr->ds + pr->K);
  }
  if (!pr->lp && !pr->ph1 && d.P) gemv_n(st, pr->n, pr->n, 1.0, d.P, d.ldp, pr->dx, 0.0, pr->Pdx);
}

// one pass over all slacks for candidates k0..k0+63: mask + barrier sums into pr->mask/sums
void candidate_pass(ipm_problem* pr, const double* x, double alpha0, double beta) {
  hipStream_t st = S(pr);
  if (!pr->socp) {
    ls_lin(st, pr->S, pr->Sbar, pr->s0, pr->ds, alpha0, beta, pr->pmask, pr->psum);
    ls_fold(st, ls_lin_blocks(pr->S), pr->pmask, pr->psum, pr->mask, pr->sums);
  } else {
    const double* shp = pr->ph1 ? x + pr->n : nullptr;
    const double* dshp = pr->ph1 ? pr->dx + pr->n : nullptr;
    ls_cone(st, pr->sv, pr->lhs0, pr->dlhs, pr->rhs0, pr->drhs, shp, dshp, alpha0, beta, pr->pmask, pr->psum);
    int64_t nb = pr->K;
    if (pr->nbb > 0) {
      ls_lin(st, pr->nbb, pr->nbb, pr->s0 + pr->K, pr->ds + pr->K, alpha0, beta, pr->pmask + pr->K,
             pr->psum + pr->K * NCAND);
      nb += ls_lin_blocks(pr->nbb);
    }
    ls_fold(st, nb, pr->pmask, pr->psum, pr->mask, pr->sums);
  }
}

struct Readback {
  int info, info2;
  unsigned long long mask;
  double sums[NCAND];
  double sc[SC_COUNT];
};

int readback(ipm_problem* pr, Readback& r, bool want_info) {
  ipm_handle* h = pr->h;
  hipStream_t st = S(pr);
  char* hb = reinterpret_cast<char*>(h->hbuf);
  hipMemcpyAsync(hb, pr->info, RB_SCAL + SC_COUNT * sizeof(double), hipMemcpyDeviceToHost, st);
  HIPCHK(h, hipStreamSynchronize(st));
  if (h->timing) {
    float ms = 0.f;
    if (h->kkt_pending && hipEventElapsedTime(&ms, h->ev[0], h->ev[1]) == hipSuccess) {
      h->kkt_sum += ms; h->kkt_cnt++;
    }
    if (h->potrf_pending && hipEventElapsedTime(&ms, h->ev[2], h->ev[3]) == hipSuccess) {
      h->potrf_sum += ms; h->potrf_cnt++;
    }
    h->kkt_pending = h->potrf_pending = false;
  }
  std::memcpy(&r.info, hb, sizeof(int));
  std::memcpy(&r.info2, hb + 4, sizeof(int));
  int lerr;
  std::memcpy(&lerr, hb + 4 * RB_INFO_LSQ, sizeof(int));
  if (lerr) {
    hipMemsetAsync(lsq_info(pr), 0, sizeof(int), st);
    h->err = "least squares: the Jacobi eigensolver did not converge (numpy: SVD did not converge in Linear Least Squares)";
    return IPM_LINALG_NOT_CONVERGED;
  }
  if (r.info < 0 || r.info2 < 0) {
    // a Cholesky wait ran past its bound (POTRF_INFO_SPIN): the factor is garbage, not "not PD"
    hipMemsetAsync(pr->info, 0, 2 * sizeof(int), st);
    h->err = "Cholesky: a wait inside the factorization ran past its wall-clock bound (info " +
             std::to_string(std::min(r.info, r.info2)) + "); the Newton step was discarded";
    return IPM_HIP_ERROR;
  }
  int derr;
  std::memcpy(&derr, hb + 4 * RB_INFO_TRSV_ERR, sizeof(int));
  if (derr) {
    // a backward-solve chain producer missed the spin bound: the step in dx is not a solve result
    hipMemsetAsync(trsv_err(pr), 0, sizeof(unsigned), st);
    h->err = "backward solve: a chain producer did not publish within the spin bound (device error word " +
             std::to_string(derr) + "); the Newton step was discarded";
    return IPM_HIP_ERROR;
  }
  if (!want_info) r.info = r.info2 = 0;
  std::memcpy(&r.mask, hb + RB_MASK, 8);
  std::memcpy(r.sums, hb + RB_SUMS, NCAND * 8);
  std::memcpy(r.sc, hb + RB_SCAL, SC_COUNT * 8);
  return IPM_OK;
}

// f(alpha) on the host from the scalar pieces (expansion of f(x + a dx))
double f_at(ipm_problem* pr, const double* sc, double a) {
  if (pr->ph1) return sc[SC_F0A] + a * sc[SC_DFA];
  if (pr->lp) return sc[SC_F0A] + a * sc[SC_DFA];
  double v = 0.0;
  if (pr->d.P) v = v + 1.0 / 2.0 * ((sc[SC_F0A] + 2.0 * a * sc[SC_DFA]) + a * a * sc[SC_DDF]);
  if (pr->d.q) v = v + (sc[SC_F0B] + a * sc[SC_DFB]);
  return v;
}

int enqueue_scalars(ipm_problem* pr, const double* x, bool infeasible, const double* v, bool zeroed = false) {
  const ipm_problem_desc& d = pr->d;
  ReduceBatch rb{};
  int cnt = 0;
  objective_parts(pr, x, rb, cnt);
  auto add = [&](const double* a, const double* b, int64_t len, int kind, int slot) {
    rb.ops[cnt++] = ReduceOp{a, b, len, 1, 1, kind, slot};
  };
  if (pr->ph1) {
    add(pr->dx + pr->n, nullptr, 1, RED_SUM, SC_DFA);
    add(x + pr->n, nullptr, 1, RED_SUM, SC_XN);
    add(pr->dx + pr->n, nullptr, 1, RED_SUM, SC_DXN);
  } else if (pr->lp) {
    add(d.c, pr->dx, pr->n, RED_DOT, SC_DFA);
  } else {
    if (d.P) {
      add(x, pr->Pdx, pr->n, RED_DOT, SC_DFA);
      add(pr->dx, pr->Pdx, pr->n, RED_DOT, SC_DDF);
    }
    if (d.q) add(d.q, pr->dx, pr->n, RED_DOT, SC_DFB);
  }
  add(pr->g, x, pr->N, RED_DOT, SC_GX);
  add(pr->g, pr->dx, pr->N, RED_DOT, SC_GDX);
  if (pr->Sbar > 0) add(pr->s0, nullptr, pr->Sbar, RED_SUMLOG, SC_SUMLOG0);
  if (infeasible) {
    add(pr->tmpn, nullptr, pr->n, RED_SUMSQ, SC_R0A);
    add(pr->Axb, nullptr, pr->p, RED_SUMSQ, SC_R0B);
  }
  (void)v;
  if (!zeroed) fill(S(pr), pr->scal, SC_COUNT, 0.0);
  reduce(S(pr), rb, cnt, pr->scal);
  return IPM_OK;
}

}  // namespace

// symmetric expansion in place (the lower triangle mirrored into the upper; no scratch)
static int expand_full_inplace(ipm_problem* pr, double* M, int64_t n, int64_t ld) {
  sym_expand_inplace(S(pr), n, M, ld);
  return IPM_OK;
}

namespace {

// dense feasible direction on the Cholesky path; LU if use_backup.
int direction_feasible(ipm_problem* pr, double t, const ipm_newton_opts* o) {
  hipStream_t st = S(pr);
  if (pr->diag) {
    assemble_hessian(pr, t, pr->s0, false);
    inv_eps(st, pr->n, pr->hdiag, 0.0, pr->tmpn);          // 1/h
    mul(st, pr->n, pr->tmpn, pr->g, -1.0, pr->dx);          // (-1/h) * g
    hipMemsetAsync(pr->info, 0, sizeof(int), st);
    return IPM_OK;
  }
  assemble_hessian(pr, t, pr->s0, o->use_psd_condition != 0);
  if (!pr->use_backup) {
    // Cholesky of the bordered [[H, -g], [-g^T, big]]: its last row is y = L^-1 (-g) (the forward
    // solve of NewtonSolver.py:287-299 / cho_solve), then one backward solve L^T dx = y
    ipm_handle* h = pr->h;
    if (h->timing) { hipEventRecord(h->ev[2], st); h->potrf_pending = true; }
    // bordered: columns 0..N-1 only (row N of L is the forward-solved right-hand side); the row
    // N = -g itself is written by the launch that zeroes the factorization's control words
    {
      BorderJob bj;
      bj.N = pr->N;
      bj.H = pr->H;
      bj.ldh = pr->ldh;
      bj.g = pr->g;
      bj.scale = -1.0;
      const int rcb = potrf_step(pr, st, pr->N + 1, pr->H, pr->ldh, pr->info, pr->pws, pr->N, &bj);
      if (rcb) return rcb;
    }
    if (h->timing) hipEventRecord(h->ev[3], st);
    trsv_lower_t(st, pr->N, pr->H, pr->ldh, pr->H + pr->N, pr->ldh, pr->dx, pr->ctl, pr->xinv, trsv_err(pr));
  } else if (!pr->lu) {
    // np_lstsq, and the Cholesky-failure backup (NewtonSolver.py:212-227, 334-341):
    // lstsq(H, -g, rcond=None), minimum norm on the eigenvectors of H
    lincomb(st, pr->N, -1.0, pr->g, 0.0, nullptr, pr->dx);
    int rc = expand_full_inplace(pr, pr->H, pr->N, pr->ldh);
    if (rc) return rc;
    double* lw = pr->lsw;
    if (!lw) { pr->h->err = "no least-squares workspace"; return IPM_HIP_ERROR; }
    if (lstsq_sym_factor(&pr->h->rb, st, pr->N, pr->H, pr->ldh, lw, lsq_info(pr)) ||
        lstsq_sym_apply(&pr->h->rb, st, pr->N, 1, pr->H, pr->ldh, pr->dx, 1, lw)) {
      pr->h->err = "least-squares library call failed";
      return IPM_HIP_ERROR;
    }
    hipMemsetAsync(pr->info, 0, sizeof(int), st);
  } else {
    // np_solve / direct: LU with partial pivoting (NewtonSolver.py:230-247, 344-361)
    lincomb(st, pr->N, -1.0, pr->g, 0.0, nullptr, pr->dx);
    int rc = expand_full_inplace(pr, pr->H, pr->N, pr->ldh);
    if (rc) return rc;
    double* lw = scratch(pr->h, (size_t)getrf_ws_doubles(pr->N) * sizeof(double));
    if (!lw) { pr->h->err = "scratch alloc failed"; return IPM_HIP_ERROR; }
    getrf(st, pr->N, pr->H, pr->ldh, pr->piv, pr->info, lw);
    getrs(st, pr->N, 1, pr->H, pr->ldh, pr->piv, pr->dx, 1);
    hipMemsetAsync(pr->info, 0, sizeof(int), st);
  }
  return IPM_OK;
}

// np_lstsq block elimination (NewtonSolverInfeasibleStart.py:279-316): four lstsq calls, three of
// them on A11 = H (one eigendecomposition shared), one on S = A H^+ A^T.  Expects H assembled and
// pr->Axb = A x - b; writes dx, dv.
int direction_infeasible_lstsq(ipm_problem* pr, const double* v) {
  const ipm_problem_desc& d = pr->d;
  hipStream_t st = S(pr);
  const int64_t n = pr->n, p = pr->p, lds = schur_ld(p);
  int rc = expand_full_inplace(pr, pr->H, n, pr->ldh);
  if (rc) return rc;
  // the problem's least-squares workspace: H's factor, S's factor, a p x p temporary
  const int64_t wh = lstsq_ws_doubles(n, p), ws = lstsq_ws_doubles(p, 1);
  double* lw = pr->lsw;
  if (!lw) { pr->h->err = "no least-squares workspace"; return IPM_HIP_ERROR; }
  double* lws = lw + wh;
  double* stmp = lws + ws;
  void** rb = &pr->h->rb;
  bool bad = lstsq_sym_factor(rb, st, n, pr->H, pr->ldh, lw, lsq_info(pr)) != 0;
  // Y = H^+ A^T (n x p row-major), hg = H^+ g
  copy(st, pr->Ybuf, d.AT, n * p);
  bad = bad || lstsq_sym_apply(rb, st, n, p, pr->H, pr->ldh, pr->Ybuf, p, lw) != 0;
  copy(st, pr->tmpn, pr->g, n);
  bad = bad || lstsq_sym_apply(rb, st, n, 1, pr->H, pr->ldh, pr->tmpn, 1, lw) != 0;
  // S = A Y, w = S^+ (b2 - A hg)
  SyrkEpi e;
  syrk_lower(st, p, n, 1.0, d.AT, p, pr->Ybuf, p, nullptr, 0.0, pr->Sbuf, lds, e);
  sym_lower_to_full(st, p, pr->Sbuf, lds, stmp, lds);
  copy(st, pr->Sbuf, stmp, p * lds);
  bad = bad || lstsq_sym_factor(rb, st, p, pr->Sbuf, lds, lws, lsq_info(pr)) != 0;
  gemv_n(st, p, n, 1.0, d.A, d.lda, pr->tmpn, 0.0, pr->r2);
  lincomb(st, p, 1.0, pr->Axb, -1.0, pr->r2, pr->wv);
  bad = bad || lstsq_sym_apply(rb, st, p, 1, pr->Sbuf, lds, pr->wv, 1, lws) != 0;
  // dx = -H^+ (g + A^T w)
  gemv_t(st, p, n, 1.0, d.A, d.lda, pr->wv, nullptr, 0.0, pr->ATdv, pr->part, pr->part_elems);
  lincomb(st, n, -1.0, pr->g, -1.0, pr->ATdv, pr->dx);
  bad = bad || lstsq_sym_apply(rb, st, n, 1, pr->H, pr->ldh, pr->dx, 1, lw) != 0;
  if (bad) { pr->h->err = "least-squares library call failed"; return IPM_HIP_ERROR; }
  lincomb(st, p, 1.0, pr->wv, -1.0, v, pr->dv);
  hipMemsetAsync(pr->info, 0, 2 * sizeof(int), st);
  return IPM_OK;
}

// infeasible-start block elimination (NewtonSolverInfeasibleStart.py:386-538, 774-809)
// x: current point, v: dual.  Writes dx, dv, and Axb (= A x - b).
int direction_infeasible(ipm_problem* pr, const double* x, const double* v, double t,
                         const ipm_newton_opts* o, bool* lin_alg_error) {
  const ipm_problem_desc& d = pr->d;
  hipStream_t st = S(pr);
  const int64_t n = pr->n, p = pr->p;
  *lin_alg_error = false;
  // b2 = A x - b
  gemv_n(st, p, n, 1.0, d.A, d.lda, x, 0.0, pr->Axb);
  lincomb(st, p, 1.0, pr->Axb, -1.0, d.b, pr->Axb);
  if (pr->diag) {
    assemble_hessian(pr, t, pr->s0, false);
    inv_eps(st, n, pr->hdiag, 0.0, pr->tmpn);  // Hi = 1/h
    // S = A diag(Hi) A^T   (lower, column-major ld = schur_ld(p))
    const int64_t lds = schur_ld(p);
    SyrkEpi e;
    syrk_lower(st, p, n, 1.0, d.AT, p, nullptr, 0, pr->tmpn, 0.0, pr->Sbuf, lds, e);
    double* lw = nullptr;
    if (pr->lsq) {
      // NewtonSolverNPLstSqDiagonalInfeasibleStart (NewtonSolverInfeasibleStart.py:692-724): w = lstsq(S, r)
      int rc = expand_full_inplace(pr, pr->Sbuf, p, lds);
      if (rc) return rc;
      lw = pr->lsw;
      if (!lw) { pr->h->err = "no least-squares workspace"; return IPM_HIP_ERROR; }
      if (lstsq_sym_factor(&pr->h->rb, st, p, pr->Sbuf, lds, lw, lsq_info(pr))) {
        pr->h->err = "least-squares library call failed";
        return IPM_HIP_ERROR;
      }
    } else {
      potrf_lower(st, p, pr->Sbuf, lds, pr->info, pr->pws);
    }
    // r = b2 - A (Hi * g)
    mul(st, n, pr->tmpn, pr->g, 1.0, pr->hxs);
    gemv_n(st, p, n, 1.0, d.A, d.lda, pr->hxs, 0.0, pr->r2);
    lincomb(st, p, 1.0, pr->Axb, -1.0, pr->r2, pr->wv);
    if (pr->lsq) {
      if (lstsq_sym_apply(&pr->h->rb, st, p, 1, pr->Sbuf, lds, pr->wv, 1, lw)) {
        pr->h->err = "least-squares library call failed";
        return IPM_HIP_ERROR;
      }
      hipMemsetAsync(pr->info, 0, sizeof(int), st);
    } else {
      potrs_lower(st, p, 1, pr->Sbuf, lds, pr->wv, 1, pr->Wp, pr->ctl);
    }
    // dx = (-Hi) * (g + A^T w)
    gemv_t(st, p, n, 1.0, d.A, d.lda, pr->wv, nullptr, 0.0, pr->ATdv, pr->part, pr->part_elems);
    lincomb(st, n, 1.0, pr->g, 1.0, pr->ATdv, pr->hxs);
    mul(st, n, pr->tmpn, pr->hxs, -1.0, pr->dx);
    lincomb(st, p, 1.0, pr->wv, -1.0, v, pr->dv);
    return IPM_OK;
  }
  assemble_hessian(pr, t, pr->s0, o->use_psd_condition != 0);
  const int64_t lds = schur_ld(p);
  if (!pr->use_backup) {
    potrf_lower_fused(st, pr->N, pr->H, pr->ldh, pr->info, pr->pws);
    // Y = H^-1 A^T  (n x p row-major); hg = H^-1 g
    copy(st, pr->Ybuf, d.AT, n * p);
    if (p >= 32 && n >= 128) {
      // many right-hand sides: 128-row blocks on MFMA GEMMs (handle scratch, grown on demand)
      double* bw = scratch(pr->h, (size_t)potrs_blocked_ws_doubles(n, p) * sizeof(double));
      if (!bw) { pr->h->err = "scratch alloc failed"; return IPM_HIP_ERROR; }
      potrs_blocked(st, n, p, pr->H, pr->ldh, pr->Ybuf, p, bw);
    } else {
      potrs_lower(st, n, p, pr->H, pr->ldh, pr->Ybuf, p, pr->W2, pr->ctl);
    }
    copy(st, pr->tmpn, pr->g, n);
    potrs_lower(st, n, 1, pr->H, pr->ldh, pr->tmpn, 1, pr->W2, pr->ctl, pr->xinv, trsv_err(pr));
    // S = A Y: the reference factors np.matmul(A, A11_inv_AT) with scipy's cho_factor, which reads
    // the UPPER triangle (lower=False; NewtonSolverInfeasibleStart.py:473-477).  A Y is not exactly
    // symmetric in rounding (Y carries the solve's errors), so the factored triangle is the one the
    // reference reads: the lower triangle of (A Y)^T, i.e. X = Y, Y = A^T in the SYRK form
    SyrkEpi e;
    syrk_lower(st, p, n, 1.0, pr->Ybuf, p, d.AT, p, nullptr, 0.0, pr->Sbuf, lds, e);
    potrf_lower(st, p, pr->Sbuf, lds, pr->info + 1, pr->pws);
    // w = S^-1 (b2 - A hg)
    gemv_n(st, p, n, 1.0, d.A, d.lda, pr->tmpn, 0.0, pr->r2);
    lincomb(st, p, 1.0, pr->Axb, -1.0, pr->r2, pr->wv);
    potrs_lower(st, p, 1, pr->Sbuf, lds, pr->wv, 1, pr->Wp, pr->ctl);
    // dx = -H^-1 (g + A^T w)
    gemv_t(st, p, n, 1.0, d.A, d.lda, pr->wv, nullptr, 0.0, pr->ATdv, pr->part, pr->part_elems);
    lincomb(st, n, -1.0, pr->g, -1.0, pr->ATdv, pr->dx);
    potrs_lower(st, n, 1, pr->H, pr->ldh, pr->dx, 1, pr->W2, pr->ctl, pr->xinv, trsv_err(pr));
    lincomb(st, p, 1.0, pr->wv, -1.0, v, pr->dv);
    return IPM_OK;
  }
  if (pr->lsq) return direction_infeasible_lstsq(pr, v);
  // LU fallback: four np.linalg.solve (NewtonSolverInfeasibleStart.py:513-538)
  int rc = expand_full_inplace(pr, pr->H, n, pr->ldh);
  if (rc) return rc;
  double* lw = scratch(pr->h, (size_t)getrf_ws_doubles(n) * sizeof(double));
  if (!lw) { pr->h->err = "scratch alloc failed"; return IPM_HIP_ERROR; }
  getrf(st, n, pr->H, pr->ldh, pr->piv, pr->info, lw);
  copy(st, pr->Ybuf, d.AT, n * p);
  getrs(st, n, p, pr->H, pr->ldh, pr->piv, pr->Ybuf, p);
  copy(st, pr->tmpn, pr->g, n);
  getrs(st, n, 1, pr->H, pr->ldh, pr->piv, pr->tmpn, 1);
  // S = A Y in FULL, both triangles computed (np.matmul(A, A11_inv_AT), :527-529): the LU reads
  // all of it, and at large t the asymmetry of A Y (the solve's rounding in Y) steers the step.
  // A mirrored lower triangle instead moved lp_eq_ineq's x* by 2.9e-3 (oracle emulation, DESIGN
  // §2.1), where the reference's own LU-rounding spread is 5e-8.  Column-major: S(i, j) at
  // Sbuf[j * lds + i] = sum_k A^T[k][i] Y[k][j]
  gemm_kk(st, p, p, n, d.AT, p, pr->Ybuf, p, pr->Sbuf, lds);
  getrf(st, p, pr->Sbuf, lds, pr->pivp, pr->info + 1, lw);
  gemv_n(st, p, n, 1.0, d.A, d.lda, pr->tmpn, 0.0, pr->r2);
  lincomb(st, p, 1.0, pr->Axb, -1.0, pr->r2, pr->wv);
  getrs(st, p, 1, pr->Sbuf, lds, pr->pivp, pr->wv, 1);
  gemv_t(st, p, n, 1.0, d.A, d.lda, pr->wv, nullptr, 0.0, pr->ATdv, pr->part, pr->part_elems);
  lincomb(st, n, -1.0, pr->g, -1.0, pr->ATdv, pr->dx);
  getrs(st, n, 1, pr->H, pr->ldh, pr->piv, pr->dx, 1);
  lincomb(st, p, 1.0, pr->wv, -1.0, v, pr->dv);
  hipMemsetAsync(pr->info, 0, 2 * sizeof(int), st);
  return IPM_OK;
}

// gradient at x with fresh slacks into pr->g (also leaves go, Px, pieces).  hess_add >= 0 (the
// feasible-start loop, LP / QP / LP phase 1 with C rows): the fused path -- C x and P x in one
// GEMV launch, slacks / inverses / w / go / dvec in one elementwise launch, C^T inv with the
// gradient combine in its second stage: 4 launches instead of 10, every value bitwise the same
// (IPM_FUSED_GRAD=0: the separate kernels)
void gradient_at(ipm_problem* pr, const double* x, double t, double hess_add = -1.0) {
  const char* efg = getenv("IPM_FUSED_GRAD");   // (read per call: a test compares both paths)
  const bool fused_on = !(efg && efg[0] == '0');
  const ipm_problem_desc& d = pr->d;
  if (fused_on && hess_add >= 0.0 && !pr->socp && pr->m > 0 && !pr->diag) {
    hipStream_t st = S(pr);
    const bool qpP = !pr->ph1 && !pr->lp && d.P;
    if (qpP) gemv_n2(st, pr->n, x, pr->m, d.C, d.ldc, pr->Cx, pr->n, d.P, d.ldp, pr->Px);
    else gemv_n(st, pr->m, pr->n, 1.0, d.C, d.ldc, x, 0.0, pr->Cx);
    LinPieces a;
    a.n = pr->n;
    a.m = pr->m;
    a.d = d.d;
    a.Cx = pr->Cx;
    a.lb = d.lb;
    a.ub = d.ub;
    a.x = x;
    a.shp = pr->ph1 ? x + pr->n : nullptr;
    a.t = t;
    a.ph1 = pr->ph1;
    a.s = pr->s0;
    a.inv = pr->inv;
    a.w = pr->w;
    if (!pr->ph1) {
      a.go = pr->go;
      if (pr->lp) a.c = d.c;
      else { a.Px = d.P ? pr->Px : nullptr; a.q = d.q; }
    }
    a.dvec = pr->dvec;
    a.add = hess_add;
    lin_pieces(st, a);
    gemv_t_grad(st, pr->m, pr->n, d.C, d.ldc, pr->inv, pr->ct, pr->part, pr->part_elems, pr->ph1 ? nullptr : pr->go,
                inv_lb(pr), inv_ub(pr), pr->ph1, pr->g);
    if (pr->ph1) {
      ReduceBatch rb{};
      rb.ops[0] = ReduceOp{pr->inv, nullptr, pr->Sbar, 1, 1, RED_SUM, SC_SUMINV};
      reduce(st, rb, 1, pr->scal);
      t_minus(st, t, pr->scal + SC_SUMINV, pr->g + pr->n);
    }
    pr->pieces_valid = true;
    pr->hess_pre = true;
    pr->hess_add = hess_add;
    return;
  }
  compute_slacks(pr, x, pr->s0, pr->lhs0, pr->rhs0);
  objective_grad(pr, x, t);
  barrier_pieces(pr, pr->s0, pr->lhs0, pr->rhs0);
  assemble_gradient(pr, t, pr->s0, pr->g);
}

}  // namespace

extern "C" int ipm_newton_solve(ipm_problem* pr, double* x, double t, double* v, const ipm_newton_opts* o,
                                ipm_newton_result* res) {
  if (!pr || !x || !o || !res) return IPM_INVALID_ARG;
  if (pr->eq && !v) return IPM_INVALID_ARG;
  ipm_handle* h = pr->h;
  hipStream_t st = S(pr);
  std::memset(res, 0, sizeof(*res));
  HostTable tab;
  tab.build(o->beta, 256);
  const int K = o->update_slacks_every;
  Readback rb{};
  int64_t backtracks = 0;
  int it = 0;
  double stat = 0.0;
  bool stat_valid = false;

  auto finish = [&](int iters, bool ok, bool have_stat, double st_v) {
    res->iters = iters;
    res->success = ok ? 1 : 0;
    res->stat_valid = have_stat ? 1 : 0;
    res->stat = st_v;
    res->use_backup = pr->use_backup ? 1 : 0;
    res->backtracks = backtracks;
    // leave the oracle state fresh at x (the reference's final fm.update_x(x))
    copy(st, pr->xe, x, pr->N);
    compute_slacks(pr, x, pr->s0, pr->lhs0, pr->rhs0);
    hipError_t e = hipStreamSynchronize(st);
    if (e != hipSuccess) { h->err = hipGetErrorString(e); return IPM_HIP_ERROR; }
    return IPM_OK;
  };
  // an eigensolve that did not converge (np.linalg.lstsq raising LinAlgError inside the reference's
  // Newton loop) ends this Newton solve as a failure, as the reference's try/except does
  // (NewtonSolver.py:148-155, NewtonSolverInfeasibleStart.py:161-164); other errors propagate
  auto bail = [&](int rc) {
    if (rc != IPM_LINALG_NOT_CONVERGED) return rc;
    const int r2 = finish(it + 1, false, stat_valid, stat);
    res->linalg_error = 1;
    return r2;
  };

  for (it = 0; it < o->max_iters; ++it) {
    gradient_at(pr, x, t, pr->eq ? -1.0 : (o->use_psd_condition != 0 ? 1e-9 : 0.0));
    if (!pr->eq) {
      // ------------------------------------------------ feasible start (NewtonSolver.py)
      int rc = direction_feasible(pr, t, o);
      if (rc) return bail(rc);
      const bool zs = !pr->socp;
      prep_linesearch_dirs(pr, zs);
      enqueue_scalars(pr, x, false, nullptr, zs);
      int64_t k0 = 0;
      candidate_pass(pr, x, tab.alpha[0], o->beta);
      rc = readback(pr, rb, true);
      if (rc) return bail(rc);
      if (rb.info != 0 && !pr->use_backup && !pr->diag) {
        // Cholesky failed: permanent LU fallback (Q9); H must be rebuilt (potrf overwrote it)
        pr->use_backup = true;
        rc = direction_feasible(pr, t, o);
        if (rc) return bail(rc);
        prep_linesearch_dirs(pr);
        enqueue_scalars(pr, x, false, nullptr);
        candidate_pass(pr, x, tab.alpha[0], o->beta);
        rc = readback(pr, rb, false);
        if (rc) return bail(rc);
      }
      const double fx = t * f_at(pr, rb.sc, 0.0) - rb.sc[SC_SUMLOG0];
      const double gc = rb.sc[SC_GX];
      // (a) the 64-candidate table: slacks s0 + a ds, f(x + a dx) from its expansion, decisions
      //     replayed on the host (default)
      auto table_step = [&](double* out) -> int {
        int64_t kd = -1, kstuck = -1;
        for (int64_t k = 0;; ++k) {
          tab.build(o->beta, k + 1);
          if (k > 0 && tab.alpha[k] < STEP_FLOOR) { kstuck = k; break; }
          if (k >= k0 + NCAND) {
            k0 = k;
            candidate_pass(pr, x, tab.alpha[k0], o->beta);
            const int rc2 = readback(pr, rb, false);
            if (rc2) return rc2;
          }
          ++backtracks;
          if (rb.mask & (1ull << (k - k0))) { kd = k; break; }
        }
        if (kd < 0) {
          *out = tab.alpha[kstuck];
          return IPM_OK;
        }
        // Armijo loop with the reference's lag (Q3) and stale slacks (Q2)
        int64_t ks = kd, kx = kd, kslack = kd;
        int attempt = 0;
        for (;;) {
          if (kslack < k0 || kslack >= k0 + NCAND) {
            k0 = kslack;
            tab.build(o->beta, k0 + NCAND);
            candidate_pass(pr, x, tab.alpha[k0], o->beta);
            const int rc2 = readback(pr, rb, false);
            if (rc2) return rc2;
          }
          const double psi = t * f_at(pr, rb.sc, tab.alpha[kx]) - rb.sums[kslack - k0];
          if (!(psi > fx + o->alpha * tab.alpha[ks] * gc)) break;
          ++attempt;
          ++backtracks;
          const int64_t knext = ks;
          if (tab.alpha[ks] < STEP_FLOOR) break;
          ++ks;
          tab.build(o->beta, ks + 1);
          kx = knext;
          if (K > 0 && attempt % K == K - 1) kslack = knext;
        }
        *out = tab.alpha[ks];
        return IPM_OK;
      };
      // (b) reference-exact (IPM_LS_EXACT): every trial point next_x = x + a dx is formed, its
      //     slacks come from a fresh d - C next_x GEMV when the reference refreshes them, and
      //     f(next_x) is evaluated directly (P next_x GEMV) -- NewtonSolver.py:165-206 step by step,
      //     one device->host copy per trial
      auto exact_step = [&](double* out) -> int {
        const ipm_problem_desc& dd = pr->d;
        double f_cur = 0.0, sl_cur = 0.0;
        bool feas = true;
        auto eval_at = [&](double a, bool fresh) -> int {
          lincomb(st, pr->N, 1.0, x, a, pr->dx, pr->xd);
          ReduceBatch rbt{};
          int cnt = 0;
          if (!pr->lp && !pr->ph1 && dd.P) gemv_n(st, pr->n, pr->n, 1.0, dd.P, dd.ldp, pr->xd, 0.0, pr->Px);
          objective_parts(pr, pr->xd, rbt, cnt);
          fill(st, pr->scal, SC_COUNT, 0.0);
          reduce(st, rbt, cnt, pr->scal);
          if (fresh && pr->S > 0) {
            compute_slacks(pr, pr->xd, pr->sdv, nullptr, nullptr);
            // candidate 0 of a pass with alpha0 = 0 is the fresh slack vector itself
            ls_lin(st, pr->S, pr->Sbar, pr->sdv, pr->ds, 0.0, o->beta, pr->pmask, pr->psum);
            ls_fold(st, ls_lin_blocks(pr->S), pr->pmask, pr->psum, pr->mask, pr->sums);
          }
          Readback r{};
          const int rc2 = readback(pr, r, false);
          if (rc2) return rc2;
          f_cur = f_at(pr, r.sc, 0.0);
          if (fresh) {
            feas = pr->S > 0 ? (r.mask & 1ull) != 0 : true;
            sl_cur = pr->S > 0 ? r.sums[0] : 0.0;
          }
          return IPM_OK;
        };
        double a = 1.0;
        int rc2 = eval_at(a, true);
        if (rc2) return rc2;
        while (!feas) {                              // domain loop (NewtonSolver.py:172-183)
          a *= o->beta;
          if (a < STEP_FLOOR) { *out = a; return IPM_OK; }
          rc2 = eval_at(a, true);
          if (rc2) return rc2;
        }
        int attempt = 0;                             // Armijo loop (NewtonSolver.py:185-202)
        while (t * f_cur - sl_cur > fx + o->alpha * a * gc) {
          ++attempt;
          const double a_pt = a;                     // next_x = x + a dx BEFORE a *= beta (Q3)
          if (a < STEP_FLOOR) { *out = a; return IPM_OK; }
          a *= o->beta;
          rc2 = eval_at(a_pt, K > 0 && attempt % K == K - 1);
          if (rc2) return rc2;
        }
        *out = a;
        return IPM_OK;
      };
      double step = 0.0;
      const int lsm = o->linesearch_mode;
      if (lsm != IPM_LS_EXACT) {
        rc = table_step(&step);
        if (rc) return bail(rc);
      }
      if (lsm == IPM_LS_EXACT || lsm == IPM_LS_COMPARE) {
        if (pr->socp) {
          h->err = "reference-exact line search: LP / QP / phase 1 only";
          return IPM_NOT_SUPPORTED;
        }
        const Readback rb0 = rb;                     // g.x, g.dx, x[n], dx[n] of this step
        double se = 0.0;
        rc = exact_step(&se);
        if (rc) return bail(rc);
        rb = rb0;
        if (lsm == IPM_LS_COMPARE) {
          ++res->ls_compared;
          if (se != step) ++res->ls_flips;
        }
        step = se;
      }
      axpy(st, pr->N, step, pr->dx, x);
      res->last_step = step;
      if (o->trace && it < o->trace_cap) { o->trace[2 * it] = step; o->trace[2 * it + 1] = -rb.sc[SC_GDX] / 2; }
      if (pr->ph1 && o->phase1_flag) {
        const double xn = rb.sc[SC_XN] + step * rb.sc[SC_DXN];
        if (xn < -o->phase1_tol) return finish(it + 1, true, false, 0.0);
      }
      const double nd = -rb.sc[SC_GDX] / 2;
      stat = nd;
      stat_valid = true;
      if (step < STEP_FLOOR) return finish(it + 1, false, true, nd);
      if (nd < o->eps) return finish(it + 1, true, true, nd);
    } else {
      // ------------------------------------------------ infeasible start
      bool lae = false;
      int rc = direction_infeasible(pr, x, v, t, o, &lae);
      if (rc) return bail(rc);
      prep_linesearch_dirs(pr);
      // r = ||[g + A^T v ; A x - b]||  (pieces)
      const ipm_problem_desc& d = pr->d;
      gemv_t(st, pr->p, pr->n, 1.0, d.A, d.lda, v, nullptr, 0.0, pr->ATv, pr->part, pr->part_elems);
      lincomb(st, pr->n, 1.0, pr->g, 1.0, pr->ATv, pr->tmpn);
      gemv_t(st, pr->p, pr->n, 1.0, d.A, d.lda, pr->dv, nullptr, 0.0, pr->ATdv, pr->part, pr->part_elems);
      gemv_n(st, pr->p, pr->n, 1.0, d.A, d.lda, pr->dx, 0.0, pr->Adx);
      enqueue_scalars(pr, x, true, v);
      int64_t k0 = 0;
      candidate_pass(pr, x, tab.alpha[0], o->beta);
      rc = readback(pr, rb, true);
      if (rc) return bail(rc);
      // info[0]: H, info[1]: S (Cholesky paths)
      const int info2 = rb.info2;
      if (pr->diag) {
        if (rb.info != 0) {
          // the diagonal class has no try/except: LinAlgError propagates to solve() -> fail
          return finish(it + 1, false, stat_valid, stat);
        }
      } else if ((rb.info != 0 || info2 != 0) && !pr->use_backup) {
        pr->use_backup = true;
        rc = direction_infeasible(pr, x, v, t, o, &lae);
        if (rc) return bail(rc);
        prep_linesearch_dirs(pr);
        gemv_t(st, pr->p, pr->n, 1.0, d.A, d.lda, v, nullptr, 0.0, pr->ATv, pr->part, pr->part_elems);
        lincomb(st, pr->n, 1.0, pr->g, 1.0, pr->ATv, pr->tmpn);
        gemv_t(st, pr->p, pr->n, 1.0, d.A, d.lda, pr->dv, nullptr, 0.0, pr->ATdv, pr->part, pr->part_elems);
        gemv_n(st, pr->p, pr->n, 1.0, d.A, d.lda, pr->dx, 0.0, pr->Adx);
        enqueue_scalars(pr, x, true, v);
        candidate_pass(pr, x, tab.alpha[0], o->beta);
        rc = readback(pr, rb, false);
        if (rc) return bail(rc);
      }
      const double r0 = std::sqrt(rb.sc[SC_R0A] + rb.sc[SC_R0B]);
      int64_t kd = -1, kstuck = -1;
      for (int64_t k = 0;; ++k) {
        tab.build(o->beta, k + 1);
        if (k > 0 && tab.alpha[k] < STEP_FLOOR) { kstuck = k; break; }
        if (k >= k0 + NCAND) {
          k0 = k;
          candidate_pass(pr, x, tab.alpha[k0], o->beta);
          rc = readback(pr, rb, false);
          if (rc) return bail(rc);
        }
        ++backtracks;
        if (rb.mask & (1ull << (k - k0))) { kd = k; break; }
      }
      double step;
      bool have_rn = false;
      double rn = 0.0;
      if (kd < 0) {
        step = tab.alpha[kstuck];
      } else {
        // slack state at the domain point: x_d = x + a_d dx, fresh slacks
        auto barrier_at = [&](int64_t kk) {
          lincomb(st, pr->N, 1.0, x, tab.alpha[kk], pr->dx, pr->xd);
          compute_slacks(pr, pr->xd, pr->sdv, pr->lhsd, pr->rhsd);
          barrier_pieces(pr, pr->sdv, pr->lhsd, pr->rhsd);
          assemble_barrier_grad(pr, pr->gb);
        };
        barrier_at(kd);
        ResidView rv{};
        rv.n = pr->n; rv.p = pr->p; rv.t = t;
        rv.c = pr->lp ? d.c : nullptr;
        rv.Px = (!pr->lp && d.P) ? pr->Px : nullptr;
        rv.Pdx = (!pr->lp && d.P) ? pr->Pdx : nullptr;
        rv.q = pr->lp ? nullptr : d.q;
        rv.B = pr->gb; rv.ATv = pr->ATv; rv.ATdv = pr->ATdv; rv.Axb = pr->Axb; rv.Adx = pr->Adx;
        // next_grad in the reference's association (see ResidView): the pieces barrier_at left
        rv.blb = inv_lb(pr);
        rv.bub = inv_ub(pr);
        rv.ct = (pr->m > 0 || pr->socp) ? pr->ct : nullptr;
        rv.ct_first = pr->socp;
        auto resid_pass = [&](int64_t kk0) -> int {
          tab.build(o->beta, kk0 + NCAND);
          ls_resid(st, rv, tab.alpha[kk0], o->beta, pr->pmask, pr->psum);
          ls_fold(st, ls_resid_blocks(rv.n, rv.p), pr->pmask, pr->psum, pr->mask, pr->sums);
          return readback(pr, rb, false);
        };
        int64_t rk0 = kd;
        rc = resid_pass(rk0);
        if (rc) return bail(rc);
        int64_t ks = kd;
        rn = std::sqrt(rb.sums[0]);
        int attempt = 0;
        while (rn > (1 - o->alpha * tab.alpha[ks]) * r0) {
          ++attempt;
          ++backtracks;
          ++ks;
          tab.build(o->beta, ks + 1);
          if (tab.alpha[ks] < STEP_FLOOR) break;
          const bool refresh = K > 0 && attempt % K == K - 1;
          if (refresh) {
            barrier_at(ks);
            rk0 = ks;
            rc = resid_pass(rk0);
            if (rc) return bail(rc);
          } else if (ks >= rk0 + NCAND) {
            rk0 = ks;
            rc = resid_pass(rk0);
            if (rc) return bail(rc);
          }
          rn = std::sqrt(rb.sums[ks - rk0]);
        }
        have_rn = true;
        step = tab.alpha[ks];
      }
      axpy(st, pr->N, step, pr->dx, x);
      axpy(st, pr->p, step, pr->dv, v);
      res->last_step = step;
      if (o->trace && it < o->trace_cap) { o->trace[2 * it] = step; o->trace[2 * it + 1] = have_rn ? rn : NAN; }
      stat = rn;
      stat_valid = have_rn;
      if (step < STEP_FLOOR) return finish(it + 1, false, have_rn, rn);
      if (have_rn && rn < o->eps) return finish(it + 1, true, true, rn);
    }
  }
  return finish(it, false, stat_valid, stat);
}
