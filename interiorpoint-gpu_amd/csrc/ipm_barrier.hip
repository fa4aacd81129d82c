// Barrier-oracle and line-search kernels (HBM-bound, elementwise / segmented reductions).
//
// Restates on device the per-iteration vector work of FunctionManager.py (slacks, barrier
// value, gradient pieces, SOCP cone terms) and of the two backtracking searches
// (NewtonSolver.py:157-206, NewtonSolverInfeasibleStart.py:170-273).  Instead of one GEMV
// + one device->host sync per trial point (the reference's loops), every candidate step
// alpha_k = beta^k (k = k0 .. k0+63) is evaluated in ONE pass over the slacks: a 64-bit
// feasibility mask and 64 barrier sums (or 64 residual norms) come back in one copy.
#include "ipm_barrier.h"

#include <algorithm>

namespace ipm {

static inline int64_t cdiv(int64_t a, int64_t b) { return (a + b - 1) / b; }

constexpr double EPS_LOG = 1e-15;   // FunctionManager.py:223-227, 244-246
constexpr double EPS_CONE = 1e-12;  // FunctionManager.py:1084-1098, 1136, 1152-1154

// ------------------------------------------------------------------------------- slacks
// LP / QP / LP-phase-1 slacks:  [sh + d - Cx | sh + ub - x | sh + x - lb]
// (FunctionManager.py:118-149 with sh = 0; :427-449 with sh = s)
__global__ void k_slacks_lin(int64_t n, int64_t m, const double* __restrict__ d,
                             const double* __restrict__ Cx, const double* __restrict__ lb,
                             const double* __restrict__ ub, const double* __restrict__ x,
                             const double* __restrict__ shp, double* __restrict__ s) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nub = ub ? n : 0, nlb = lb ? n : 0;
  if (e >= m + nub + nlb) return;
  if (shp) {
    const double sh = *shp;
    if (e < m) s[e] = (sh + d[e]) - Cx[e];
    else if (e < m + nub) { const int64_t i = e - m; s[e] = (sh + ub[i]) - x[i]; }
    else { const int64_t i = e - m - nub; s[e] = (sh + x[i]) - lb[i]; }
  } else {
    if (e < m) s[e] = d[e] - Cx[e];
    else if (e < m + nub) { const int64_t i = e - m; s[e] = ub[i] - x[i]; }
    else { const int64_t i = e - m - nub; s[e] = x[i] - lb[i]; }
  }
}

void slacks_lin(hipStream_t st, int64_t n, int64_t m, const double* d, const double* Cx, const double* lb,
                const double* ub, const double* x, const double* shp, double* s) {
  const int64_t tot = m + (ub ? n : 0) + (lb ? n : 0);
  if (tot > 0)
    hipLaunchKernelGGL(k_slacks_lin, dim3(cdiv(tot, 256)), dim3(256), 0, st, n, m, d, Cx, lb, ub, x, shp, s);
}

// f(v) helpers ----------------------------------------------------------------------
__global__ void k_inv_eps(int64_t len, const double* __restrict__ s, double eps, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < len) out[e] = 1.0 / (s[e] + eps);
}
void inv_eps(hipStream_t st, int64_t len, const double* s, double eps, double* out) {
  if (len > 0) hipLaunchKernelGGL(k_inv_eps, dim3(cdiv(len, 256)), dim3(256), 0, st, len, s, eps, out);
}

__global__ void k_sq(int64_t len, const double* __restrict__ a, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < len) { const double v = a[e]; out[e] = v * v; }
}
void square(hipStream_t st, int64_t len, const double* a, double* out) {
  if (len > 0) hipLaunchKernelGGL(k_sq, dim3(cdiv(len, 256)), dim3(256), 0, st, len, a, out);
}

// objective gradient:  go = t * c (LP)   |   go = (Px + q) * t (QP/SOCP; q, Px may be null)
__global__ void k_objgrad(int64_t n, double t, const double* __restrict__ c, const double* __restrict__ Px,
                          const double* __restrict__ q, double* __restrict__ go) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  if (c) { go[i] = t * c[i]; return; }
  double v = Px ? Px[i] : 0.0;
  if (q) v = v + q[i];
  go[i] = v * t;
}
void objgrad(hipStream_t st, int64_t n, double t, const double* c, const double* Px, const double* q,
             double* go) {
  if (n > 0) hipLaunchKernelGGL(k_objgrad, dim3(cdiv(n, 256)), dim3(256), 0, st, n, t, c, Px, q, go);
}

// g = ((go - blb) + bub) + ct          (LP/QP order, FunctionManager.py:248-263)
// g = (((go) + ct) - blb) + bub         (ct_first: SOCP / phase-1 order, :526-535, :1080-1100)
__global__ void k_grad_combine(int64_t n, const double* __restrict__ go, const double* __restrict__ blb,
                               const double* __restrict__ bub, const double* __restrict__ ct, bool ct_first,
                               double* __restrict__ g) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double v;
  if (ct_first) {
    v = go ? go[i] : 0.0;
    if (ct) v = go ? v + ct[i] : ct[i];
    if (blb) v = v - blb[i];
    if (bub) v = v + bub[i];
  } else {
    v = go ? go[i] : 0.0;
    if (blb) v = v - blb[i];
    if (bub) v = v + bub[i];
    if (ct) v = v + ct[i];
  }
  g[i] = v;
}
void grad_combine(hipStream_t st, int64_t n, const double* go, const double* blb, const double* bub,
                  const double* ct, bool ct_first, double* g) {
  if (n > 0)
    hipLaunchKernelGGL(k_grad_combine, dim3(cdiv(n, 256)), dim3(256), 0, st, n, go, blb, bub, ct, ct_first, g);
}

// dvec = a^2 + b^2 (a or b may be null), optionally plus psd
__global__ void k_dvec(int64_t n, const double* __restrict__ a, const double* __restrict__ b, double add,
                       double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double v = 0.0;
  if (a) v = v + a[i] * a[i];
  if (b) v = v + b[i] * b[i];
  out[i] = v + add;
}
void dvec_sq(hipStream_t st, int64_t n, const double* a, const double* b, double add, double* out) {
  if (n > 0) hipLaunchKernelGGL(k_dvec, dim3(cdiv(n, 256)), dim3(256), 0, st, n, a, b, add, out);
}

// dvec for 1/s^2 WITHOUT eps (LP/QP bound Hessian terms, FunctionManager.py:320-322)
__global__ void k_dvec_inv(int64_t n, const double* __restrict__ slb, const double* __restrict__ sub,
                           double add, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double v = 0.0;
  if (slb) { const double r = 1.0 / slb[i]; v = v + r * r; }
  if (sub) { const double r = 1.0 / sub[i]; v = v + r * r; }
  out[i] = v + add;
}
void dvec_inv_sq(hipStream_t st, int64_t n, const double* slb, const double* sub, double add, double* out) {
  if (n > 0) hipLaunchKernelGGL(k_dvec_inv, dim3(cdiv(n, 256)), dim3(256), 0, st, n, slb, sub, add, out);
}

// SOCP bound Hessian term 1/(s + 1e-12)^2 (FunctionManager.py:1148-1154)
__global__ void k_dvec_inv_eps(int64_t n, const double* __restrict__ slb, const double* __restrict__ sub,
                               double add, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double v = 0.0;
  if (slb) { const double r = 1.0 / (slb[i] + EPS_CONE); v = v + r * r; }
  if (sub) { const double r = 1.0 / (sub[i] + EPS_CONE); v = v + r * r; }
  out[i] = v + add;
}
void dvec_inv_eps_sq(hipStream_t st, int64_t n, const double* slb, const double* sub, double add, double* out) {
  if (n > 0) hipLaunchKernelGGL(k_dvec_inv_eps, dim3(cdiv(n, 256)), dim3(256), 0, st, n, slb, sub, add, out);
}

// dst[i] += scale[c] * a[c][i]^2 for diagonal cones (AtA_cache = diag(a^2), FunctionManager.py:878-886)
__global__ void k_dvec_diag_cones(int64_t n, int64_t Kd, const double* __restrict__ Ad,
                                  const int64_t* __restrict__ cid, const double* __restrict__ coef,
                                  double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double v = out[i];
  for (int64_t c = 0; c < Kd; ++c) {
    const double a = Ad[c * n + i];
    v = v + coef[cid[c]] * (a * a);
  }
  out[i] = v;
}
void dvec_diag_cones(hipStream_t st, int64_t n, int64_t Kd, const double* Ad, const int64_t* cid,
                     const double* coef, double* out) {
  if (n > 0 && Kd > 0)
    hipLaunchKernelGGL(k_dvec_diag_cones, dim3(cdiv(n, 256)), dim3(256), 0, st, n, Kd, Ad, cid, coef, out);
}

// x = x + a * dx  (separate multiply and add, as NumPy's `x += step * xstep`)
__global__ void k_axpy(int64_t n, double a, const double* __restrict__ dx, double* __restrict__ x) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) { const double t = a * dx[i]; x[i] = x[i] + t; }
}
void axpy(hipStream_t st, int64_t n, double a, const double* dx, double* x) {
  if (n > 0) hipLaunchKernelGGL(k_axpy, dim3(cdiv(n, 256)), dim3(256), 0, st, n, a, dx, x);
}

// out = a * u + b * v   (v may be null)
__global__ void k_lincomb(int64_t n, double a, const double* __restrict__ u, double b,
                          const double* __restrict__ v, double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  double r = a * u[i];
  if (v) r = r + b * v[i];
  out[i] = r;
}
void lincomb(hipStream_t st, int64_t n, double a, const double* u, double b, const double* v, double* out) {
  if (n > 0) hipLaunchKernelGGL(k_lincomb, dim3(cdiv(n, 256)), dim3(256), 0, st, n, a, u, b, v, out);
}

// out = u * v  (elementwise), optional negate
__global__ void k_mul(int64_t n, const double* __restrict__ u, const double* __restrict__ v, double sgn,
                      double* __restrict__ out) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) out[i] = (sgn * u[i]) * v[i];
}
void mul(hipStream_t st, int64_t n, const double* u, const double* v, double sgn, double* out) {
  if (n > 0) hipLaunchKernelGGL(k_mul, dim3(cdiv(n, 256)), dim3(256), 0, st, n, u, v, sgn, out);
}

// The LP-family gradient pieces at x in one pass (given Cx, and Px for a QP), each value formed
// exactly as the separate kernels form it: slacks (k_slacks_lin), inv = 1/(s + 1e-15) (k_inv_eps),
// w = inv^2 over the C rows (k_sq), go (k_objgrad, not in phase 1), and -- when dvec != null --
// the Hessian's diagonal vector (phase 1: k_dvec of the bound inverses, else k_dvec_inv of the
// bound slacks) plus `add`.  Thread e: C row e (e < m) and variable e (e < n).
__global__ void k_lin_pieces(LinPieces a) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t n = a.n, m = a.m, nub = a.ub ? n : 0;
  const double sh = a.shp ? *a.shp : 0.0;
  if (e < m) {
    const double se = a.shp ? (sh + a.d[e]) - a.Cx[e] : a.d[e] - a.Cx[e];
    a.s[e] = se;
    const double iv = 1.0 / (se + 1e-15);
    a.inv[e] = iv;
    if (a.w) a.w[e] = iv * iv;
  }
  if (e < n) {
    double su = 0.0, sl = 0.0, iu = 0.0, il = 0.0;
    if (a.ub) {
      su = a.shp ? (sh + a.ub[e]) - a.x[e] : a.ub[e] - a.x[e];
      a.s[m + e] = su;
      iu = 1.0 / (su + 1e-15);
      a.inv[m + e] = iu;
    }
    if (a.lb) {
      sl = a.shp ? (sh + a.x[e]) - a.lb[e] : a.x[e] - a.lb[e];
      a.s[m + nub + e] = sl;
      il = 1.0 / (sl + 1e-15);
      a.inv[m + nub + e] = il;
    }
    if (a.go) {
      if (a.c) {
        a.go[e] = a.t * a.c[e];
      } else {
        double v = a.Px ? a.Px[e] : 0.0;
        if (a.q) v = v + a.q[e];
        a.go[e] = v * a.t;
      }
    }
    if (a.dvec) {
      double v = 0.0;
      if (a.ph1) {
        if (a.lb) v = v + il * il;
        if (a.ub) v = v + iu * iu;
      } else {
        if (a.lb) { const double r = 1.0 / sl; v = v + r * r; }
        if (a.ub) { const double r = 1.0 / su; v = v + r * r; }
      }
      a.dvec[e] = v + a.add;
    }
  }
}
void lin_pieces(hipStream_t st, const LinPieces& a) {
  const int64_t tot = std::max(a.m, a.n);
  if (tot > 0) hipLaunchKernelGGL(k_lin_pieces, dim3(cdiv(tot, 256)), dim3(256), 0, st, a);
}

// slack directions for the LP family: ds = [dsh - Cdx | dsh - dx | dsh + dx]
__global__ void k_dslacks_lin(int64_t n, int64_t m, const double* __restrict__ Cdx, bool has_lb, bool has_ub,
                              const double* __restrict__ dx, const double* __restrict__ dshp,
                              double* __restrict__ ds, double* __restrict__ zero, int nzero) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (zero && e < nzero) zero[e] = 0.0;   // (the scalar slots of the next reduction: fill() folded in)
  const int64_t nub = has_ub ? n : 0, nlb = has_lb ? n : 0;
  if (e >= m + nub + nlb) return;
  const double dsh = dshp ? *dshp : 0.0;
  double v;
  if (e < m) v = -Cdx[e];
  else if (e < m + nub) v = -dx[e - m];
  else v = dx[e - m - nub];
  ds[e] = dshp ? dsh + v : v;
}
void dslacks_lin(hipStream_t st, int64_t n, int64_t m, const double* Cdx, bool has_lb, bool has_ub,
                 const double* dx, const double* dshp, double* ds, double* zero, int nzero) {
  const int64_t tot = std::max<int64_t>(m + (has_ub ? n : 0) + (has_lb ? n : 0), zero ? nzero : 0);
  if (tot > 0)
    hipLaunchKernelGGL(k_dslacks_lin, dim3(cdiv(tot, 256)), dim3(256), 0, st, n, m, Cdx, has_lb, has_ub, dx,
                       dshp, ds, zero, nzero);
}

// s_out = s0 + a * ds   (a from a device scalar if ap != null)
__global__ void k_slack_at(int64_t len, const double* __restrict__ s0, const double* __restrict__ ds,
                           double a, double* __restrict__ out) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e < len) out[e] = s0[e] + a * ds[e];
}
void slack_at(hipStream_t st, int64_t len, const double* s0, const double* ds, double a, double* out) {
  if (len > 0) hipLaunchKernelGGL(k_slack_at, dim3(cdiv(len, 256)), dim3(256), 0, st, len, s0, ds, a, out);
}

// --------------------------------------------------------------------- scalar reductions
// one workgroup per descriptor; deterministic fixed-order reduction
__global__ __launch_bounds__(1024) void k_reduce(ReduceBatch batch, double* __restrict__ out) {
  const ReduceOp op = batch.ops[blockIdx.x];
  __shared__ double red[16];
  double acc = 0.0;
  for (int64_t i = threadIdx.x; i < op.len; i += 1024) {
    const double a = op.a[i * op.sa];
    double v;
    switch (op.kind) {
      case RED_DOT: v = a * op.b[i * op.sb]; break;
      case RED_SUM: v = a; break;
      case RED_SUMSQ: v = a * a; break;
      case RED_SUMLOG: v = log(a + EPS_LOG); break;
      case RED_SUMINV: v = 1.0 / (a + EPS_LOG); break;
      case RED_SUMINV2: { const double r = 1.0 / (a + EPS_LOG); v = r * r; } break;
      default: v = 0.0;
    }
    acc += v;
  }
  const double s = block_sum(acc, red);
  if (threadIdx.x == 0) out[op.slot] = s;
}
void reduce(hipStream_t st, const ReduceBatch& b, int count, double* out) {
  if (count > 0) hipLaunchKernelGGL(k_reduce, dim3(count), dim3(1024), 0, st, b, out);
}

// --------------------------------------------------------------------------- SOCP cones
// lhs_r = (X x)_r + b_r for dense rows; lhs(diag cone c) = a_c * x + b_c.
// rhs_i = c_i.x + d_i  (or d_i, or c_i.x) from Xx rows [R, R+K).
// sdst[i] = rhs^2 - ||lhs||^2 (+ sh);  also bounds and the appended rhs block.
// One workgroup per cone.  (FunctionManager.py:933-994, 1258-1262)
__global__ __launch_bounds__(256) void k_cone_slacks(SocpView v, const double* __restrict__ Xx,
                                                     const double* __restrict__ x,
                                                     const double* __restrict__ shp,
                                                     double* __restrict__ lhs, double* __restrict__ rhs,
                                                     double* __restrict__ s) {
  __shared__ double red[16];
  const int64_t i = blockIdx.x;
  const int64_t r0 = v.off[i], r1 = v.off[i + 1];
  double acc = 0.0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
    double l = Xx[r];
    if (v.cb) l = l + v.cb[r];
    lhs[r] = l;
    acc += l * l;
  }
  const int64_t dc = v.dslot[i];  // diagonal cone slot or -1
  if (dc >= 0) {
    for (int64_t j = threadIdx.x; j < v.n; j += 256) {
      double l = v.Ad[dc * v.n + j] * x[j];
      if (v.bd) l = l + v.bd[dc * v.n + j];
      lhs[v.R + dc * v.n + j] = l;
      acc += l * l;
    }
  }
  const double ss = block_sum(acc, red);
  if (threadIdx.x == 0) {
    double rh;
    if (v.has_c) {
      rh = Xx[v.R + i];
      if (v.cd) rh = rh + v.cd[i];
    } else {
      rh = v.cd ? v.cd[i] : 0.0;
    }
    rhs[i] = rh;
    double sv = rh * rh - ss;
    if (shp) sv = sv + *shp;
    s[i] = sv;
    s[v.K + v.nbnd + i] = rh;  // appended rhs block (domain only, Q15)
  }
}

__global__ void k_bound_slacks(int64_t n, int64_t off, const double* __restrict__ lb,
                               const double* __restrict__ ub, const double* __restrict__ x,
                               const double* __restrict__ shp, double* __restrict__ s) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t nub = ub ? n : 0, nlb = lb ? n : 0;
  if (e >= nub + nlb) return;
  double v;
  if (e < nub) v = ub[e] - x[e];
  else v = x[e - nub] - lb[e - nub];
  if (shp) v = v + *shp;
  s[off + e] = v;
}

void cone_slacks(hipStream_t st, const SocpView& v, const double* Xx, const double* x, const double* lb,
                 const double* ub, const double* shp, double* lhs, double* rhs, double* s) {
  hipLaunchKernelGGL(k_cone_slacks, dim3(v.K), dim3(256), 0, st, v, Xx, x, shp, lhs, rhs, s);
  const int64_t nb = v.nbnd;
  if (nb > 0)
    hipLaunchKernelGGL(k_bound_slacks, dim3(cdiv(nb, 256)), dim3(256), 0, st, v.n, v.K, lb, ub, x, shp, s);
}

// per-cone coefficients: SOCP coef_i = 2/(s_i + 1e-12); SOCP phase 1 coef_i = 2 * inv_i with
// inv_i = 1/(sigma_i + 1e-15) (FunctionManager.py:1130-1140, 1405-1415)
__global__ void k_cone_coef(int64_t K, const double* __restrict__ s, bool phase1, double* __restrict__ coef,
                            double* __restrict__ invs) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= K) return;
  if (phase1) {
    const double iv = 1.0 / (s[i] + EPS_LOG);
    invs[i] = iv;
    coef[i] = 2.0 * iv;
  } else {
    coef[i] = 2.0 / (s[i] + EPS_CONE);
  }
}
void cone_coef(hipStream_t st, int64_t K, const double* s, bool phase1, double* coef, double* invs) {
  if (K > 0) hipLaunchKernelGGL(k_cone_coef, dim3(cdiv(K, 256)), dim3(256), 0, st, K, s, phase1, coef, invs);
}

// SYRK row weights: dense rows of cone i and row R+i (c_i) get coef_i; G rows get 1
__global__ void k_cone_rowweights(SocpView v, const double* __restrict__ coef, double* __restrict__ w) {
  const int64_t r = (int64_t)blockIdx.x * 256 + threadIdx.x;
  const int64_t rows = v.R + 2 * v.K;
  if (r >= rows) return;
  if (r < v.R) w[r] = coef[v.rowcone[r]];
  else if (r < v.R + v.K) w[r] = coef[r - v.R];
  else w[r] = 1.0;
}
void cone_rowweights(hipStream_t st, const SocpView& v, const double* coef, double* w) {
  const int64_t rows = v.R + 2 * v.K;
  hipLaunchKernelGGL(k_cone_rowweights, dim3(cdiv(rows, 256)), dim3(256), 0, st, v, coef, w);
}

// G_i[j] = (sum_{r in cone i} lhs_r X[r][j] (+ a_i[j] lhs_i[j]) - c_i[j] rhs_i) * coef_i
// written to X rows [R + K + i]  (FunctionManager.py:1115-1140)
__global__ __launch_bounds__(256) void k_cone_grows(SocpView v, const double* __restrict__ lhs,
                                                    const double* __restrict__ rhs,
                                                    const double* __restrict__ coef) {
  const int64_t i = blockIdx.y;
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= v.n) return;
  const int64_t r0 = v.off[i], r1 = v.off[i + 1];
  double acc = 0.0;
  for (int64_t r = r0; r < r1; ++r) acc = fma(v.X[r * v.ldx + j], lhs[r], acc);
  const int64_t dc = v.dslot[i];
  if (dc >= 0) acc = acc + v.Ad[dc * v.n + j] * lhs[v.R + dc * v.n + j];
  if (v.has_c) acc = acc - v.X[(v.R + i) * v.ldx + j] * rhs[i];
  v.X[(v.R + v.K + i) * v.ldx + j] = acc * coef[i];
}
void cone_grows(hipStream_t st, const SocpView& v, const double* lhs, const double* rhs, const double* coef) {
  if (v.K <= 0) return;
  hipLaunchKernelGGL(k_cone_grows, dim3(cdiv(v.n, 256), v.K), dim3(256), 0, st, v, lhs, rhs, coef);
}

// ------------------------------------------------------------------- line-search passes
// LP family: trial slacks s0 + alpha_k ds.  Per workgroup partials:
//   pmask[blk] = AND over elements of the 64-bit "!(v<0)" mask,
//   psum[blk*64 + k] = sum log(v + 1e-15) over elements with barrier flag.
// alpha_k = alpha0 * beta^k by repeated multiplication (bit-identical to the host table).
__device__ __forceinline__ void lane_reduce_store(double (&vals)[64], unsigned long long mask,
                                                  unsigned long long* __restrict__ pmask,
                                                  double* __restrict__ psum) {
  __shared__ double red[64][4];
  __shared__ unsigned long long mred[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    const double s = wave_sum(vals[k]);
    if (lane == 0) red[k][wv] = s;
  }
  unsigned long long mm = mask;
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mm &= __shfl_xor(mm, off, 64);
  if (lane == 0) mred[wv] = mm;
  __syncthreads();
  if (threadIdx.x < 64) {
    const int k = threadIdx.x;
    psum[(int64_t)blockIdx.x * 64 + k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
  }
  if (threadIdx.x == 0) pmask[blockIdx.x] = ((mred[0] & mred[1]) & mred[2]) & mred[3];
}

// 64 slacks per workgroup; wave w evaluates candidates 16w .. 16w+15 for all 64 (lane = slack),
// so a wave sum is a candidate's partial and no cross-wave reduction is needed.  4x the
// workgroups of a one-slack-per-thread form (the 64 logs per slack were the cost).
constexpr int LS_EPB = 64;   // slacks per workgroup
__global__ __launch_bounds__(256) void k_ls_lin(int64_t len, int64_t bar_len, const double* __restrict__ s0,
                                                const double* __restrict__ ds, double alpha0, double beta,
                                                unsigned long long* __restrict__ pmask,
                                                double* __restrict__ psum) {
  __shared__ unsigned long long mq[4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int64_t e = (int64_t)blockIdx.x * LS_EPB + lane;
  double a = alpha0;
  for (int q = 0; q < 16 * wv; ++q) a = a * beta;   // alpha_{16w}, as the host table forms it
  double vals[16];
  unsigned mask = 0xFFFFu;
  if (e < len) {
    const double a0 = s0[e], d = ds[e];
    const bool bar = e < bar_len;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const double v = a0 + a * d;
      if (v < 0.0) mask &= ~(1u << k);
      vals[k] = bar ? log(v + EPS_LOG) : 0.0;
      a = a * beta;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 16; ++k) vals[k] = 0.0;
  }
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const double sm = wave_sum(vals[k]);
    if (lane == 0) psum[(int64_t)blockIdx.x * 64 + 16 * wv + k] = sm;
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) mask &= (unsigned)__shfl_xor((int)mask, off, 64);
  if (lane == 0) mq[wv] = (unsigned long long)(mask & 0xFFFFu) << (16 * wv);
  __syncthreads();
  if (threadIdx.x == 0) pmask[blockIdx.x] = ((mq[0] | mq[1]) | mq[2]) | mq[3];
}

// SOCP cones: one workgroup per cone.  lhs_r(a) = lhs_r + a dlhs_r; rhs(a) = rhs + a drhs;
// sigma = rhs(a)^2 - ||lhs(a)||^2 (+ sh + a dsh for phase 1); domain also needs rhs(a) >= 0.
__global__ __launch_bounds__(256) void k_ls_cone(SocpView v, const double* __restrict__ lhs,
                                                 const double* __restrict__ dlhs,
                                                 const double* __restrict__ rhs,
                                                 const double* __restrict__ drhs,
                                                 const double* __restrict__ shp,
                                                 const double* __restrict__ dshp, double alpha0,
                                                 double beta, unsigned long long* __restrict__ pmask,
                                                 double* __restrict__ psum) {
  const int64_t i = blockIdx.x;
  const int64_t r0 = v.off[i], r1 = v.off[i + 1];
  double vals[64];
#pragma unroll
  for (int k = 0; k < 64; ++k) vals[k] = 0.0;
  for (int64_t r = r0 + threadIdx.x; r < r1; r += 256) {
    const double l = lhs[r], dl = dlhs[r];
    double a = alpha0;
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      const double t = l + a * dl;
      vals[k] += t * t;
      a = a * beta;
    }
  }
  const int64_t dc = v.dslot[i];
  if (dc >= 0) {
    for (int64_t j = threadIdx.x; j < v.n; j += 256) {
      const double l = lhs[v.R + dc * v.n + j], dl = dlhs[v.R + dc * v.n + j];
      double a = alpha0;
#pragma unroll
      for (int k = 0; k < 64; ++k) {
        const double t = l + a * dl;
        vals[k] += t * t;
        a = a * beta;
      }
    }
  }
  // block-reduce the 64 squared norms
  __shared__ double red[64][4];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int k = 0; k < 64; ++k) {
    const double s = wave_sum(vals[k]);
    if (lane == 0) red[k][wv] = s;
  }
  __syncthreads();
  __shared__ double nrm[64];
  if (threadIdx.x < 64) {
    const int k = threadIdx.x;
    nrm[k] = ((red[k][0] + red[k][1]) + red[k][2]) + red[k][3];
  }
  __syncthreads();
  if (threadIdx.x < 64) {
    const int k = threadIdx.x;
    double a = alpha0;
    for (int q = 0; q < k; ++q) a = a * beta;
    const double rh = rhs[i] + a * drhs[i];
    double sg = rh * rh - nrm[k];
    if (shp) sg = sg + (*shp + a * *dshp);
    const bool ok = !(sg < 0.0) && !(rh < 0.0);
    const unsigned long long bit = ok ? (1ull << k) : 0ull;
    // gather the mask: each lane k contributes its bit
    unsigned long long m = bit;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) m |= __shfl_xor(m, off, 64);
    psum[(int64_t)blockIdx.x * 64 + k] = log(sg + EPS_LOG);
    if (k == 0) pmask[blockIdx.x] = m;
  }
}

// final fold of partials (fixed order): 16 groups of 64 threads each sum a contiguous range of
// partials in order (loads batched), then the group sums are added in group order
__global__ __launch_bounds__(1024) void k_ls_fold(int64_t nblk, const unsigned long long* __restrict__ pmask,
                                                  const double* __restrict__ psum,
                                                  unsigned long long* __restrict__ mask_out,
                                                  double* __restrict__ sum_out) {
  __shared__ double red[16][64];
  __shared__ unsigned long long mred[16];
  const int k = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int64_t chunk = (nblk + 15) / 16, b0 = g * chunk, b1 = min(nblk, b0 + chunk);
  double s = 0.0;
  int64_t b = b0;
  for (; b + 8 <= b1; b += 8) {
    double v[8];
#pragma unroll
    for (int q = 0; q < 8; ++q) v[q] = psum[(b + q) * 64 + k];
#pragma unroll
    for (int q = 0; q < 8; ++q) s += v[q];
  }
  for (; b < b1; ++b) s += psum[b * 64 + k];
  red[g][k] = s;
  unsigned long long m = ~0ull;
  for (int64_t c = b0 + k; c < b1; c += 64) m &= pmask[c];
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) m &= (unsigned long long)__shfl_xor((long long)m, off, 64);
  if (k == 0) mred[g] = m;
  __syncthreads();
  if (g == 0) {
    double t = 0.0;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][k];
    sum_out[k] = t;
    if (k == 0) {
      unsigned long long mm = ~0ull;
#pragma unroll
      for (int q = 0; q < 16; ++q) mm &= mred[q];
      *mask_out = mm;
    }
  }
}

int64_t ls_lin_blocks(int64_t len) { return std::max<int64_t>(1, cdiv(len, LS_EPB)); }

void ls_lin(hipStream_t st, int64_t len, int64_t bar_len, const double* s0, const double* ds, double alpha0,
            double beta, unsigned long long* pmask, double* psum) {
  const int64_t nb = ls_lin_blocks(len);
  hipLaunchKernelGGL(k_ls_lin, dim3(nb), dim3(256), 0, st, len, bar_len, s0, ds, alpha0, beta, pmask, psum);
}

void ls_cone(hipStream_t st, const SocpView& v, const double* lhs, const double* dlhs, const double* rhs,
             const double* drhs, const double* shp, const double* dshp, double alpha0, double beta,
             unsigned long long* pmask, double* psum) {
  hipLaunchKernelGGL(k_ls_cone, dim3(v.K), dim3(256), 0, st, v, lhs, dlhs, rhs, drhs, shp, dshp, alpha0, beta,
                     pmask, psum);
}

void ls_fold(hipStream_t st, int64_t nblk, const unsigned long long* pmask, const double* psum,
             unsigned long long* mask_out, double* sum_out) {
  hipLaunchKernelGGL(k_ls_fold, dim3(1), dim3(1024), 0, st, nblk, pmask, psum, mask_out, sum_out);
}

// infeasible-start residual candidates (NewtonSolverInfeasibleStart.py:209-269):
//   dual_e(a)   = ((((Px_e + a Pdx_e) + q_e) * t  or  t c_e)  + B_e) + ATv_e + a ATdv_e
//   primal_j(a) = Axb_j + a Adx_j
//   psum[blk*64+k] = partial sum of squares
__global__ __launch_bounds__(256) void k_ls_resid(ResidView v, double alpha0, double beta,
                                                  unsigned long long* __restrict__ pmask,
                                                  double* __restrict__ psum) {
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  double vals[64];
  if (e < v.n) {
    const double Px = v.Px ? v.Px[e] : 0.0, Pdx = v.Pdx ? v.Pdx[e] : 0.0, q = v.q ? v.q[e] : 0.0;
    const bool pieces = v.blb || v.bub || v.ct;
    const double B = pieces ? 0.0 : v.B[e], atv = v.ATv[e], atdv = v.ATdv[e];
    const double blb = v.blb ? v.blb[e] : 0.0, bub = v.bub ? v.bub[e] : 0.0, ct = v.ct ? v.ct[e] : 0.0;
    const double tc = v.c ? v.t * v.c[e] : 0.0;
    double a = alpha0;
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      double go;
      if (v.c) go = tc;
      else {
        double px = Px;
        if (v.Pdx) px = Px + a * Pdx;
        go = (px + q) * v.t;
      }
      double g;
      if (!pieces) {
        g = go + B;
      } else if (v.ct_first) {
        g = go;
        if (v.ct) g = g + ct;
        if (v.blb) g = g - blb;
        if (v.bub) g = g + bub;
      } else {
        g = go;
        if (v.blb) g = g - blb;
        if (v.bub) g = g + bub;
        if (v.ct) g = g + ct;
      }
      const double r = (g + atv) + a * atdv;
      vals[k] = r * r;
      a = a * beta;
    }
  } else if (e < v.n + v.p) {
    const int64_t j = e - v.n;
    const double axb = v.Axb[j], adx = v.Adx[j];
    double a = alpha0;
#pragma unroll
    for (int k = 0; k < 64; ++k) {
      const double r = axb + a * adx;
      vals[k] = r * r;
      a = a * beta;
    }
  } else {
#pragma unroll
    for (int k = 0; k < 64; ++k) vals[k] = 0.0;
  }
  lane_reduce_store(vals, ~0ull, pmask, psum);
}
int64_t ls_resid_blocks(int64_t n, int64_t p) { return std::max<int64_t>(1, cdiv(n + p, 256)); }
void ls_resid(hipStream_t st, const ResidView& v, double alpha0, double beta, unsigned long long* pmask,
              double* psum) {
  hipLaunchKernelGGL(k_ls_resid, dim3(ls_resid_blocks(v.n, v.p)), dim3(256), 0, st, v, alpha0, beta, pmask,
                     psum);
}

// ------------------------------------------------------------ phase-1 Hessian border
// H (column-major lower, ldh) row n:  H[n][j] = hxs_j (j < n), H[n][n] = hss.
__global__ void k_border(int64_t n, double* __restrict__ H, int64_t ldh, const double* __restrict__ hxs,
                         const double* __restrict__ hssp) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j < n) H[j * ldh + n] = hxs[j];
  else if (j == n) H[n * ldh + n] = *hssp;
}
void border(hipStream_t st, int64_t n, double* H, int64_t ldh, const double* hxs, const double* hssp) {
  hipLaunchKernelGGL(k_border, dim3(cdiv(n + 1, 256)), dim3(256), 0, st, n, H, ldh, hxs, hssp);
}

// hxs = ((-ct) + lbt) - ubt   (FunctionManager.py:571-594 order: -C^T inv^2, += lb, -= ub)
__global__ void k_border_vec(int64_t n, const double* __restrict__ ct, const double* __restrict__ lbt,
                             const double* __restrict__ ubt, double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  double v = ct ? -ct[j] : 0.0;
  if (lbt) v = v + lbt[j];
  if (ubt) v = v - ubt[j];
  out[j] = v;
}
void border_vec(hipStream_t st, int64_t n, const double* ct, const double* lbt, const double* ubt, double* out) {
  if (n > 0) hipLaunchKernelGGL(k_border_vec, dim3(cdiv(n, 256)), dim3(256), 0, st, n, ct, lbt, ubt, out);
}
// the same with the bound terms squared in place (ilb[j]^2, iub[j]^2: each product rounded before
// the sum, as the separate square kernels stored it) -- one launch instead of three
__global__ void k_border_vec_sq(int64_t n, const double* __restrict__ ct, const double* __restrict__ ilb,
                                const double* __restrict__ iub, double* __restrict__ out) {
  const int64_t j = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (j >= n) return;
  double v = ct ? -ct[j] : 0.0;
  if (ilb) {
    const double a = ilb[j], a2 = a * a;
    v = v + a2;
  }
  if (iub) {
    const double b = iub[j], b2 = b * b;
    v = v - b2;
  }
  out[j] = v;
}
void border_vec_sq(hipStream_t st, int64_t n, const double* ct, const double* ilb, const double* iub, double* out) {
  if (n > 0) hipLaunchKernelGGL(k_border_vec_sq, dim3(cdiv(n, 256)), dim3(256), 0, st, n, ct, ilb, iub, out);
}

// gs = t - sumv  (device scalar)
__global__ void k_tminus(double t, const double* __restrict__ sp, double* __restrict__ out) {
  *out = t - *sp;
}
void t_minus(hipStream_t st, double t, const double* sp, double* out) {
  hipLaunchKernelGGL(k_tminus, dim3(1), dim3(1), 0, st, t, sp, out);
}

}  // namespace ipm
