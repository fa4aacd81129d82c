// fp64 MFMA tile GEMM for gfx950 (v_mfma_f64_16x16x4_f64): the KKT SYRK of the barrier
// Hessian and every GEMM-shaped update of the Cholesky factorisation.
//
//   C(i, j) (op)= sum_k  w[k] X[k][i] Y[k][j]      i < ni, j < nj, k < K
//
// Operands are "k-major": row k of X is X + k*ldx.  That covers both callers without copies:
//   * KKT assembly (FunctionManager.py:301-306, 801-805): X = Y = C (m x n row-major, k = the
//     inequality row), w = 1/(s+eps)^2;
//   * Cholesky updates: a column-major panel A(r, c) at c*lda + r is k-major with k = c.
// C is column-major (element (i, j) at j*ldc + i), i.e. the lower triangle of the row-major
// Hessian the reference builds.
//
// Workgroup = 256 threads = 2 x 2 waves, 128 x 128 output tile, each wave 64 x 64 = 4 x 4 MFMA
// tiles (64 fp64 accumulators per lane).  K is staged 16 rows at a time through two LDS
// buffers (73.7 KB -> 2 workgroups per CU) with the global loads for slab s+2 in registers
// while slab s is multiplied.  LDS rows are padded to 144 doubles: the 4 k-rows one
// ds_read_b64 touches sit 32 banks apart (conflict-free).  Full tiles run an unguarded
// load path; edge tiles (and a ragged last K slab) a guarded one -- a uniform branch.
// Triangular grids map blockIdx -> tile so that each XCD (blocks b, b+8, ...) sweeps a
// contiguous run of tile rows and keeps the shared operand panels in its own L2.
// The KKT SYRK kernels (k_mfma_gemm, _split, _streamk) run the fast loop LOOP 2 (round 6): the X
// fragments go from memory straight into the MFMA operand registers and only Y goes through LDS.
//
// Measured (MI355X): the KKT SYRK at n = 8192, K = 2048 2.19 ms = 62.8 TF/s (80 % of the fp64
// peak, MFMA busy 81 %; profiles/r6f); the Cholesky's K = 256 trailing tiles ~42-54 % (LOOP 1).
#pragma once
#include <algorithm>
#include <map>
#include <mutex>
#include <queue>
#include <tuple>
#include <type_traits>
#include <vector>

#include "ipm_common.h"

namespace ipm {

// tools/tile_lab.hip only: per-workgroup phase stamps of mfma_tile (wave 0): [0] entry, [1] slab
// loop start, [2] slab loop end, [3] epilogue stores issued, [4] stores complete (s_memtime
// cycles); [6] / [7] entry / exit on the 100 MHz clock
#ifdef IPM_TILE_STAMPS
__device__ unsigned long long ipm_tile_stamps[4096 * 8];
#define IPM_TSTAMP(k) do { if (threadIdx.x == 0 && blockIdx.x < 4096) ipm_tile_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memtime(); } while (0)
#define IPM_TSTAMPR(k) do { if (threadIdx.x == 0 && blockIdx.x < 4096) ipm_tile_stamps[blockIdx.x * 8 + (k)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define IPM_TSTAMP(k) do {} while (0)
#define IPM_TSTAMPR(k) do {} while (0)
#endif

struct GemmArgs {
  int64_t ni = 0, nj = 0, K = 0;
  const double* X = nullptr;
  int64_t ldx = 0;
  const double* Y = nullptr;
  int64_t ldy = 0;
  const double* w = nullptr;     // weight on k (applied to the X operand), may be null
  double* C = nullptr;
  int64_t ldc = 0;
  double alpha = 1.0, beta = 0.0;
  const double* P = nullptr;     // + tP * P[j*ldp + i]   (row-major symmetric P)
  int64_t ldp = 0;
  double tP = 0.0;
  const double* dvec = nullptr;  // + dvec[i] on the diagonal
  const int* info = nullptr;     // skip the launch's work when *info != 0 (failed Cholesky)
  int tri = 0;                   // lower-triangular tile grid (ni == nj), only i >= j written
  int sub = 0;                   // C -= acc  (alpha/beta/P/dvec ignored)
  int xcd_remap = 1;             // XCD-contiguous tile order (0: plain blockIdx order)
  int rowmajor = 0;              // tile L -> (L / tiles_j, L % tiles_j) (no remap): row blocks in order
  int64_t tiles_i = 0, tiles_j = 0, nblk = 0;
  int accum = 0;                 // C += alpha-free sum (accumulators start from C, P/dvec ignored)
};

// A kernel's FIRST (struct) parameter read through the kernarg segment pointer where it is used:
// as a by-value parameter every field is loaded at kernel entry by the argument lowering and the
// whole struct stays live in SGPRs across the kernel (the Cholesky kernel spilled 100-300 SGPRs to
// VGPR lanes for it).  The parameter stays declared (it defines the kernarg layout: offset 0).
// (On the GEMM kernels the same change cost the KKT SYRK 1-1.5 %, r5b: not used there.)
#define IPM_KARGS(T, name, param) \
  (void)param;                    \
  const T& name = *(const T*)__builtin_amdgcn_kernarg_segment_ptr()

// agent-coherent (sc1) element access: data handed between workgroups of ONE launch
__device__ __forceinline__ double ld_sc1(const double* p) {
  return __longlong_as_double((long long)__hip_atomic_load(
      reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ void st_sc1(double* p, double v) {
  __hip_atomic_store(reinterpret_cast<unsigned long long*>(p), (unsigned long long)__double_as_longlong(v),
                     __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// ---- bounded waits on other workgroups of the same launch (the ticketed Cholesky, its split
// trailing tiles, the persistent backward solve).  A wait gives up after a bound on the
// constant-rate GPU wall clock (s_memrealtime; 100 MHz on MI355X, the host converts microseconds
// with hipDeviceAttributeWallClockRate) and records the failure: info (if still 0) becomes
// POTRF_INFO_SPIN -- negative, never a LAPACK column -- and the launch's failure word is raised, so
// every later launch of the factorization returns at once and every other waiter of this launch
// stops waiting (it sees failw).  The host turns a negative info into IPM_HIP_ERROR: the factor is
// never used.  The bounds live in a device global read only on the slow path (after 16 polls), so
// the waits hold no extra registers in the kernels around them.  [0]: Cholesky, [1]: backward solve.
// (A static global in a header: each translation unit has its own copy.  The kernels that spin are
// all launched from ipm_blas.hip, whose copy set_spin_ticks updates on every device.)
static __device__ unsigned long long ipm_spin_ticks[2] = {100000000ull, 100000000ull};   // 1 s
__device__ __forceinline__ void spin_fail(int* info, unsigned* failw) {
  if (info) atomicCAS(info, 0, POTRF_INFO_SPIN);
  __threadfence();
  if (failw) atomicCAS(failw, 0u, 0xFFFFFFF0u);
}
// poll done() with s_sleep(SLEEP) in between; true once done, false when the bound ran out (the
// failure is recorded in info / failw, either may be null) or the launch has already failed (failw)
template <int SLEEP, int WHICH = 0, class Done>
__device__ __forceinline__ bool spin_until(int* info, unsigned* failw, Done done) {
  if (done()) return true;
  unsigned long long t0 = 0;
  for (unsigned it = 0;; ++it) {
    __builtin_amdgcn_s_sleep(SLEEP);
    if (done()) return true;
    if ((it & 15u) != 0u) continue;
    const unsigned long long now = __builtin_amdgcn_s_memrealtime();
    if (it == 0) {
      t0 = now;
      continue;
    }
    if (failw && __hip_atomic_load(failw, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u) return false;
    if (now - t0 > ipm_spin_ticks[WHICH]) {
      spin_fail(info, failw);
      return false;
    }
  }
}

// BM = 128 (4 x 4 MFMA tiles per wave) for large grids, 64 (2 x 2) when the 128-tile grid
// would leave CUs idle.  WJ = waves along j (2: 256 threads, 2 workgroups per CU; 4: 512 threads).
template <int BM_, int WJ = 2>
struct MfCfg {
  static constexpr int BM = BM_, BK = 16, NT = 128 * WJ;
  static constexpr int LD = BM + 16;        // padded LDS row: 2*LD == 32 (mod 64) dwords
  static constexpr int PT = BK * BM / NT;   // doubles per thread per slab per operand
  static constexpr int TPR = BM / PT;       // threads per slab row
  static constexpr int TWI = BM / 32;       // MFMA tiles per wave along i (2 waves)
  static constexpr int TWJ = BM / (16 * WJ);  // ... along j (WJ waves)
};

// LDS of one tile: two K slabs of each operand
// (16-byte aligned: the slab stores are ds_write_b128; with 8-byte alignment the compiler splits
//  them into ds_write2_b64 and the KKT SYRK loses ~13%)
template <int BM_, int WJ = 2>
struct alignas(16) MfSmem {
  alignas(16) double sX[2][MfCfg<BM_, WJ>::BK * MfCfg<BM_, WJ>::LD];
  alignas(16) double sY[2][MfCfg<BM_, WJ>::BK * MfCfg<BM_, WJ>::LD];
};

// One output tile (index Lw of the launch's tile space) by one workgroup of 128 * WJ threads.
// SC1OUT: the tile is stored with sc1 stores (read by other workgroups of the same launch).
// split (Cholesky trailing tiles of a launch's last round, sub tiles only): the K range is cut in
// two halves computed by two workgroups at once.  SPLIT 1 (the LOWER ticket): k in [K/2, K), the
// accumulators start at 0, the tile -X^T Y goes to the scratch tile `part` (sc1, 128 x 128
// column-major), then *pflag = 1.  SPLIT 2: k in [0, K/2) from the C tile as usual; before its
// stores it waits for *pflag and adds `part`.  Only ever waits on a lower ticket.
// SPLITADD: the non-accumulating epilogue (alpha acc + beta C + tP P + dvec) also takes the
// upper-K partial of a split tile (the KKT SYRK's split tail, k_mfma_gemm_split); a separate
// instantiation, so the Cholesky's tiles are compiled exactly as without it.
// LOOP 1: the branch-free slab loop only -- the caller guarantees a full 128-tile, whole K slabs
// (tile_fast_ok) and 16-byte operands; LOOP 0: the general loop only.  (Both loops in one
// instantiation made the register allocator spill ~2000 VGPRs.)
// LAZYC (LOOP 1, C -= X^T Y tiles with at least 16 slabs): the accumulators start at zero and the
// C tile is read one 16 x 16 MFMA block per slab (two slabs ahead of its add), so the 128 KB C read
// is spread over the K loop instead of a burst before the first MFMA (all workgroups of a round
// start together: the burst is bandwidth-bound).  C + sum(products) in another association order.
template <int BM_, bool WEIGHT, bool VEC, int WJ = 2, bool SC1OUT = false, bool SPLITADD = false, int LOOP = 0,
          int LAZYC = 0, bool CST = false>
__device__ __forceinline__ void mfma_tile(const GemmArgs& a, int64_t Lw, MfSmem<BM_, WJ>& sm, int SPLIT = 0,
                                          double* part = nullptr, unsigned* pflag = nullptr, int64_t kb = -1,
                                          int64_t ke = -1, int* sinfo = nullptr, unsigned* failw = nullptr) {
  using M = MfCfg<BM_, WJ>;
  constexpr int BM = M::BM, BK = M::BK, LD = M::LD, PT = M::PT, TPR = M::TPR, TWI = M::TWI, TWJ = M::TWJ;
  IPM_TSTAMP(0);
  IPM_TSTAMPR(6);
#ifdef IPM_TILE_STAMPS
  if (threadIdx.x == 0 && blockIdx.x < 4096)   // [5] XCC id << 32 | HW_ID
    ipm_tile_stamps[blockIdx.x * 8 + 5] = ((unsigned long long)__builtin_amdgcn_s_getreg((31 << 11) | 20) << 32) |
                                          __builtin_amdgcn_s_getreg((31 << 11) | 4);
#endif
  auto& sX = sm.sX;
  auto& sY = sm.sY;
  // ---- tile of this workgroup
  int64_t bi, bj;
  {
    int64_t L = Lw;
    const int64_t q = a.nblk >> 3;
    if (a.xcd_remap && !a.rowmajor && L < (q << 3)) L = (L & 7) * q + (L >> 3);   // XCD-contiguous tile runs
    if (a.rowmajor) {
      bi = L / a.tiles_j;
      bj = L % a.tiles_j;
    } else if (a.tri) {
      int64_t b = (int64_t)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
      while ((b + 1) * (b + 2) / 2 <= L) ++b;
      while (b * (b + 1) / 2 > L) --b;
      bi = b;
      bj = L - b * (b + 1) / 2;
    } else {
      bi = L % a.tiles_i;
      bj = L / a.tiles_i;
    }
  }
  const int64_t I0 = bi * BM, J0 = bj * BM;
  const bool full = (I0 + BM <= a.ni) && (J0 + BM <= a.nj);
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wi = wv & 1, wj = wv >> 1;
  const int sr = tid / TPR, sc = (tid % TPR) * PT;
  // SPLITADD with kb >= 0: SPLIT 1 is the K piece [kb, ke) of a stream-K tail (k_mfma_gemm_streamk)
  const bool kpiece = SPLITADD && kb >= 0;
  const int64_t kbeg = SPLIT == 1 ? (kpiece ? kb : a.K / 2) : 0;
  const double* xp = a.X + (sr + kbeg) * a.ldx + I0 + sc;
  const double* yp = a.Y + (sr + kbeg) * a.ldy + J0 + sc;
  const int64_t xstep = BK * a.ldx, ystep = BK * a.ldy;
  int kt32 = (int)a.K;
  if (SPLIT == 1) kt32 = kpiece ? (int)(ke - kb) : kt32 - kt32 / 2;
  if (SPLIT == 2) kt32 = kt32 / 2;
  const int64_t Kt = kt32;
  const int64_t nslab = (Kt + BK - 1) / BK;
  // C -= X^T Y (Cholesky updates): the accumulators start FROM the C tile (its loads overlap the
  // first slab's) and X is staged negated -- no dependent C read in the epilogue.  accum: the
  // same with C += X^T diag(w) Y.
  const bool cinit = a.sub || a.accum || (a.beta == 1.0 && a.alpha == -1.0 && !a.P && !a.dvec);
  const double xsg = (cinit && !a.accum) ? -1.0 : 1.0;
  double rx[PT], ry[PT];
  auto gload = [&](int64_t s) {
    const int64_t k = s * BK + sr;
    const double* xs = xp + s * xstep;
    const double* ys = yp + s * ystep;
    if (full && (s + 1) * BK <= Kt) {
      const double wk = WEIGHT ? a.w[kbeg + k] : 1.0;   // k counts from this piece's first row
      if (VEC) {
#pragma unroll
        for (int q = 0; q < PT / 2; ++q) {
          const double2 u = reinterpret_cast<const double2*>(xs)[q];
          const double2 v = reinterpret_cast<const double2*>(ys)[q];
          rx[2 * q] = (WEIGHT ? u.x * wk : u.x) * xsg;
          rx[2 * q + 1] = (WEIGHT ? u.y * wk : u.y) * xsg;
          ry[2 * q] = v.x;
          ry[2 * q + 1] = v.y;
        }
      } else {
#pragma unroll
        for (int q = 0; q < PT; ++q) {
          rx[q] = (WEIGHT ? xs[q] * wk : xs[q]) * xsg;
          ry[q] = ys[q];
        }
      }
    } else {
      const bool kin = k < Kt;
      const double wk = (WEIGHT && kin) ? a.w[kbeg + k] : 1.0;
#pragma unroll
      for (int q = 0; q < PT; ++q) {
        const bool xi = kin && (I0 + sc + q < a.ni), yj = kin && (J0 + sc + q < a.nj);
        rx[q] = xi ? (WEIGHT ? xs[q] * wk : xs[q]) * xsg : 0.0;
        ry[q] = yj ? ys[q] : 0.0;
      }
    }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      sX[buf][sr * LD + sc + q] = rx[q];
      sY[buf][sr * LD + sc + q] = ry[q];
    }
  };
  const int fr = lane & 15, fk = lane >> 4;
  dbl4 acc[TWJ][TWI];
#pragma unroll
  for (int u = 0; u < TWJ; ++u)
#pragma unroll
    for (int v = 0; v < TWI; ++v) acc[u][v] = dbl4{0.0, 0.0, 0.0, 0.0};
  static_assert(!LAZYC || (LOOP == 1 && !WEIGHT), "lazy C: fast loop, no weight");
  // CST (LOOP 1 full tiles, C -= X^T Y): the C tile moves through LDS in two 64-column halves --
  // each wave instruction reads / writes 4 whole 1 KB tile columns instead of 128-byte pieces
  // in four columns (the MFMA accumulator layout) -- before the first slab and after the last
  static_assert(!CST || (LOOP == 1 && !LAZYC && BM_ == 128 && WJ == 2), "staged C: 128-tile fast loop");
  constexpr int CLD = 144;   // staged column stride (doubles): 2 CLD = 32 (mod 64) dwords
  double* sCst = &sm.sX[0][0];   // sX, sY contiguous: 4 * BK * LD = 64 * CLD doubles
  static_assert(!CST || 4 * BK * LD >= 64 * CLD, "staging fits the slab buffers");
  if (CST && cinit && SPLIT == 0) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int e = tid + 256 * q, col = e >> 6, rp = e & 63;
        const double2 v = *reinterpret_cast<const double2*>(a.C + (J0 + 64 * h + col) * a.ldc + I0 + 2 * rp);
        *reinterpret_cast<double2*>(&sCst[col * CLD + 2 * rp]) = v;
      }
      __syncthreads();
      if (wj == h) {
#pragma unroll
        for (int tj = 0; tj < TWJ; ++tj)
#pragma unroll
          for (int ti = 0; ti < TWI; ++ti)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              acc[tj][ti][r] = sCst[(tj * 16 + fk + 4 * r) * CLD + wi * (BM / 2) + ti * 16 + fr];
      }
      __syncthreads();
    }
  } else if (cinit && SPLIT != 1 && !LAZYC) {
#pragma unroll
    for (int tj = 0; tj < TWJ; ++tj)
#pragma unroll
      for (int ti = 0; ti < TWI; ++ti) {
        const int64_t i = I0 + wi * (BM / 2) + ti * 16 + fr;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int64_t j = J0 + wj * (BM / WJ) + tj * 16 + fk + 4 * r;
          // (SC1OUT, the Cholesky's look-ahead tiles: the C tile is read sc1 as well -- a plain load
          // would leave the line, rows of neighbouring roles included, in this XCD's L2 until the
          // tile's sc1 stores drop it, and sc1 readers of those rows on the same XCD could be
          // served from it: r6, an unaligned leading dimension)
          acc[tj][ti][r] = (i < a.ni && j < a.nj) ? (SC1OUT ? ld_sc1(&a.C[j * a.ldc + i]) : a.C[j * a.ldc + i]) : 0.0;
        }
      }
  }
  // full 128-tiles with whole K slabs: a branch-free slab loop -- ONE basic block, so the
  // scheduler spreads the LDS reads, the LDS stores of slab s+1 and the global loads of slab s+2
  // between the MFMAs (the last loads are clamped to slab nslab-1: a harmless reload).  The weight
  // and the sign are applied when the slab goes to LDS.  tools/gemm_lab.hip (lab2): +6-9 %.
  static_assert(LOOP == 0 || (BM_ == 128 && VEC && WJ == 2), "fast loop: 128-tiles, vector loads");
  if constexpr (LAZYC) {
    // exactly 16 LAZYC slabs (K = 256 or, LAZYC 2, the block pairs' K = 512: the Cholesky's
    // trailing tiles; the caller guarantees it), fully unrolled: accumulator block q is read in
    // slab q LAZYC and added in slab (q + 2) LAZYC
    double fx[PT], fy[PT];
    auto fload = [&](int64_t s) {
      const double2* xs = reinterpret_cast<const double2*>(xp + s * xstep);
      const double2* ys = reinterpret_cast<const double2*>(yp + s * ystep);
#pragma unroll
      for (int q = 0; q < PT / 2; ++q) {
        const double2 u = xs[q], v = ys[q];
        fx[2 * q] = u.x;
        fx[2 * q + 1] = u.y;
        fy[2 * q] = v.x;
        fy[2 * q + 1] = v.y;
      }
    };
    auto fstore = [&](int buf) {
#pragma unroll
      for (int q = 0; q < PT; ++q) {
        sX[buf][sr * LD + sc + q] = fx[q] * xsg;
        sY[buf][sr * LD + sc + q] = fy[q];
      }
    };
    auto cload = [&](int q) {
      const int tj = q / TWI, ti = q % TWI;
      const int64_t i = I0 + wi * (BM / 2) + ti * 16 + fr;
      const int64_t j0 = J0 + wj * (BM / WJ) + tj * 16 + fk;
      dbl4 v;
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = a.C[(j0 + 4 * r) * a.ldc + i];
      return v;
    };
    constexpr int NS = 16, R = LAZYC > 0 ? LAZYC : 1, NSL = NS * R;
    static_assert(TWJ * TWI == NS, "one accumulator block per R slabs");
    dbl4 cq[NS];
    fload(0);
    fstore(0);
    fload(1);
    cq[0] = cload(0);
    __syncthreads();
#pragma unroll
    for (int s = 0; s < NSL; ++s) {
      const int buf = s & 1;
      const double* bx = sX[buf];
      const double* by = sY[buf];
      fstore(buf ^ 1);
      fload(s + 2 < NSL ? s + 2 : NSL - 1);
      if (s % R == 0) {
        const int q = s / R;
        if (q + 1 < NS) cq[q + 1] = cload(q + 1);
        if (q >= 2) acc[(q - 2) / TWI][(q - 2) % TWI] += cq[q - 2];
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double av[TWJ], bv[TWI];
#pragma unroll
        for (int t = 0; t < TWJ; ++t) av[t] = by[(kk * 4 + fk) * LD + wj * (BM / WJ) + t * 16 + fr];
#pragma unroll
        for (int t = 0; t < TWI; ++t) bv[t] = bx[(kk * 4 + fk) * LD + wi * (BM / 2) + t * 16 + fr];
#pragma unroll
        for (int tj = 0; tj < TWJ; ++tj)
#pragma unroll
          for (int ti = 0; ti < TWI; ++ti)
            acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tj], bv[ti], acc[tj][ti], 0, 0, 0);
      }
      __syncthreads();
    }
    acc[(NS - 2) / TWI][(NS - 2) % TWI] += cq[NS - 2];
    acc[(NS - 1) / TWI][(NS - 1) % TWI] += cq[NS - 1];
  } else if (LOOP == 1) {
    double fx[PT], fy[PT];
    double fw = 1.0;
    auto fload = [&](int64_t s) {
      const double2* xs = reinterpret_cast<const double2*>(xp + s * xstep);
      const double2* ys = reinterpret_cast<const double2*>(yp + s * ystep);
#pragma unroll
      for (int q = 0; q < PT / 2; ++q) {
        const double2 u = xs[q], v = ys[q];
        fx[2 * q] = u.x;
        fx[2 * q + 1] = u.y;
        fy[2 * q] = v.x;
        fy[2 * q + 1] = v.y;
      }
      if (WEIGHT) fw = a.w[kbeg + s * BK + sr];
    };
    auto fstore = [&](int buf) {
#pragma unroll
      for (int q = 0; q < PT; ++q) {
        sX[buf][sr * LD + sc + q] = (WEIGHT ? fx[q] * fw : fx[q]) * xsg;
        sY[buf][sr * LD + sc + q] = fy[q];
      }
    };
    fload(0);
    fstore(0);
    fload(nslab > 1 ? 1 : 0);
    __syncthreads();
    IPM_TSTAMP(1);
    for (int64_t s = 0; s < nslab; ++s) {
      const int buf = (int)(s & 1);
      const double* bx = sX[buf];
      const double* by = sY[buf];
      // slab s+1 to LDS (loaded during the previous slab; its buffer was last read before the
      // barrier) and the loads of slab s+2 issued at once: they fly under all 64 MFMAs
      fstore(buf ^ 1);
      fload(std::min<int64_t>(s + 2, nslab - 1));
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double av[TWJ], bv[TWI];
#pragma unroll
        for (int t = 0; t < TWJ; ++t) av[t] = by[(kk * 4 + fk) * LD + wj * (BM / WJ) + t * 16 + fr];
#pragma unroll
        for (int t = 0; t < TWI; ++t) bv[t] = bx[(kk * 4 + fk) * LD + wi * (BM / 2) + t * 16 + fr];
#pragma unroll
        for (int tj = 0; tj < TWJ; ++tj)
#pragma unroll
          for (int ti = 0; ti < TWI; ++ti)
            acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tj], bv[ti], acc[tj][ti], 0, 0, 0);
      }
      __syncthreads();
    }
    IPM_TSTAMP(2);
  } else if constexpr (LOOP == 2) {
    // the KKT SYRK's loop (r6): the X fragments go from memory straight into the MFMA operand
    // registers -- lane (fr, fk) of wave (wi, wj) holds X[k = 16 s + 4 kk + fk][I0 + 64 wi + 16 t +
    // fr] -- and only Y is staged through LDS (half the LDS stores and fragment reads of LOOP 1).
    // Each k-row's fragment is reloaded for the next slab right after its MFMAs are issued (one
    // slab of prefetch in the same registers).  The weight and the sign are applied to the operand
    // as LOOP 1 applies them at its LDS store: the same products, bitwise.  tools/dtv_lab.hip (r6):
    // 4.36-4.43 -> 4.12 ms on the full 8192^2 x 2048 weighted grid, 2.57-2.62 -> 2.34 ms at
    // 4096^2 x 4608 (both operands from memory: best 3.85 ms but +-5 % from run to run).
    double fy[PT];
    auto fload = [&](int64_t s) {
      const double2* ys = reinterpret_cast<const double2*>(yp + s * ystep);
#pragma unroll
      for (int q = 0; q < PT / 2; ++q) {
        const double2 v = ys[q];
        fy[2 * q] = v.x;
        fy[2 * q + 1] = v.y;
      }
    };
    auto fstore = [&](int buf) {
#pragma unroll
      for (int q = 0; q < PT; ++q) sY[buf][sr * LD + sc + q] = fy[q];
    };
    const double* xq = a.X + (kbeg + fk) * a.ldx + I0 + wi * (BM / 2) + fr;
    const double* wq = WEIGHT ? a.w + kbeg + fk : nullptr;
    double xr[BK / 4][TWI], wk[BK / 4];
    auto xload = [&](int64_t s, int kk) {
      const double* p = xq + (s * BK + kk * 4) * a.ldx;
#pragma unroll
      for (int t = 0; t < TWI; ++t) xr[kk][t] = p[t * 16];
      if (WEIGHT) wk[kk] = wq[s * BK + kk * 4];
    };
    fload(0);
    fstore(0);
    fload(nslab > 1 ? 1 : 0);
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) xload(0, kk);
    __syncthreads();
    IPM_TSTAMP(1);
    for (int64_t s = 0; s < nslab; ++s) {
      const int buf = (int)(s & 1);
      const double* by = sY[buf];
      fstore(buf ^ 1);
      fload(std::min<int64_t>(s + 2, nslab - 1));
      const int64_t sn = std::min<int64_t>(s + 1, nslab - 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double av[TWJ], bv[TWI];
#pragma unroll
        for (int t = 0; t < TWJ; ++t) av[t] = by[(kk * 4 + fk) * LD + wj * (BM / WJ) + t * 16 + fr];
#pragma unroll
        for (int t = 0; t < TWI; ++t) bv[t] = (WEIGHT ? xr[kk][t] * wk[kk] : xr[kk][t]) * xsg;
        xload(sn, kk);
#pragma unroll
        for (int tj = 0; tj < TWJ; ++tj)
#pragma unroll
          for (int ti = 0; ti < TWI; ++ti)
            acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tj], bv[ti], acc[tj][ti], 0, 0, 0);
      }
      __syncthreads();
    }
    IPM_TSTAMP(2);
  } else if constexpr (LOOP == 3) {
    // both operands' fragments from memory straight into registers: no LDS, no barriers (each
    // fragment is read by the two waves that share it; tools/dtv_lab.hip V3)
    const double* xq = a.X + (kbeg + fk) * a.ldx + I0 + wi * (BM / 2) + fr;
    const double* yq = a.Y + (kbeg + fk) * a.ldy + J0 + wj * (BM / WJ) + fr;
    const double* wq = WEIGHT ? a.w + kbeg + fk : nullptr;
    double xr[BK / 4][TWI], yr[BK / 4][TWJ], wk[BK / 4];
    auto load = [&](int64_t s, int kk) {
      const double* p = xq + (s * BK + kk * 4) * a.ldx;
      const double* q = yq + (s * BK + kk * 4) * a.ldy;
#pragma unroll
      for (int t = 0; t < TWI; ++t) xr[kk][t] = p[t * 16];
#pragma unroll
      for (int t = 0; t < TWJ; ++t) yr[kk][t] = q[t * 16];
      if (WEIGHT) wk[kk] = wq[s * BK + kk * 4];
    };
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) load(0, kk);
    for (int64_t s = 0; s < nslab; ++s) {
      const int64_t sn = std::min<int64_t>(s + 1, nslab - 1);
#pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double av[TWJ], bv[TWI];
#pragma unroll
        for (int t = 0; t < TWJ; ++t) av[t] = yr[kk][t];
#pragma unroll
        for (int t = 0; t < TWI; ++t) bv[t] = (WEIGHT ? xr[kk][t] * wk[kk] : xr[kk][t]) * xsg;
        load(sn, kk);
#pragma unroll
        for (int tj = 0; tj < TWJ; ++tj)
#pragma unroll
          for (int ti = 0; ti < TWI; ++ti)
            acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tj], bv[ti], acc[tj][ti], 0, 0, 0);
      }
    }
  } else {
    if (nslab > 0) {
      gload(0);
      sstore(0);
      if (nslab > 1) gload(1);
    }
    __syncthreads();
    for (int64_t s = 0; s < nslab; ++s) {
      const int buf = (int)(s & 1);
      const double* bx = sX[buf];
      const double* by = sY[buf];
  #pragma unroll
      for (int kk = 0; kk < BK / 4; ++kk) {
        double av[TWJ], bv[TWI];
  #pragma unroll
        for (int t = 0; t < TWJ; ++t) av[t] = by[(kk * 4 + fk) * LD + wj * (BM / WJ) + t * 16 + fr];
  #pragma unroll
        for (int t = 0; t < TWI; ++t) bv[t] = bx[(kk * 4 + fk) * LD + wi * (BM / 2) + t * 16 + fr];
  #pragma unroll
        for (int tj = 0; tj < TWJ; ++tj)
  #pragma unroll
          for (int ti = 0; ti < TWI; ++ti)
            acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tj], bv[ti], acc[tj][ti], 0, 0, 0);
      }
      if (s + 1 < nslab) {
        sstore(buf ^ 1);
        if (s + 2 < nslab) gload(s + 2);
      }
      __syncthreads();
    }
  }
  // ---- epilogue: lane holds D[j = fk + 4r][i = fr] of each 16 x 16 tile (f64 MFMA map,
  //      cdna_hip_programming.md §3) -> 16 consecutive lanes store 16 consecutive i
  if (SPLIT == 2) {
    if (tid == 0)
      spin_until<2>(sinfo, failw, [&] { return __hip_atomic_load(pflag, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0u; });
    __syncthreads();
  }
  if (CST && cinit && SPLIT == 0) {
    const bool diag = a.tri && I0 == J0;
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (wj == h) {
#pragma unroll
        for (int tj = 0; tj < TWJ; ++tj)
#pragma unroll
          for (int ti = 0; ti < TWI; ++ti)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              sCst[(tj * 16 + fk + 4 * r) * CLD + wi * (BM / 2) + ti * 16 + fr] = acc[tj][ti][r];
      }
      __syncthreads();
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        const int e = tid + 256 * q, col = e >> 6, rp = e & 63;
        const double2 v = *reinterpret_cast<const double2*>(&sCst[col * CLD + 2 * rp]);
        double* cp = a.C + (J0 + 64 * h + col) * a.ldc + I0 + 2 * rp;
        const int c = 64 * h + col;   // diagonal tile: rows >= c only
        if (!diag || 2 * rp >= c) {
          *reinterpret_cast<double2*>(cp) = v;
        } else if (2 * rp + 1 == c) {   // the pair straddles the diagonal: the lower element only
          cp[1] = v.y;
        }
      }
      if (h == 0) __syncthreads();
    }
    return;
  }
  // PRE (the GEMM / SYRK fast loops): the epilogue operands of a 16-column block (P, and C when
  // beta != 0) are loaded for all its elements before the block's first store -- vmcnt counts loads
  // and stores in issue order, so a load behind a store also waits for the store, and one element
  // at a time the KKT epilogue was ~74 us of a ~510 us tile (r6, tools/syrk_lab.hip stamps)
  constexpr bool PRE = LOOP >= 2;
#pragma unroll
  for (int tj = 0; tj < TWJ; ++tj) {
    double pp[TWI][4], pc[TWI][4];
    if constexpr (PRE) {
      if (!cinit && SPLIT != 1) {
#pragma unroll
        for (int ti = 0; ti < TWI; ++ti) {
          const int64_t i = I0 + wi * (BM / 2) + ti * 16 + fr;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const int64_t j = J0 + wj * (BM / WJ) + tj * 16 + fk + 4 * r;
            const bool ok = i < a.ni && j < a.nj && (!a.tri || i >= j);
            pp[ti][r] = (ok && a.P) ? a.P[j * a.ldp + i] : 0.0;
            pc[ti][r] = (ok && a.beta != 0.0) ? a.C[j * a.ldc + i] : 0.0;
          }
        }
      }
    }
#pragma unroll
    for (int ti = 0; ti < TWI; ++ti) {
      const int64_t i = I0 + wi * (BM / 2) + ti * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t j = J0 + wj * (BM / WJ) + tj * 16 + fk + 4 * r;
        if (SPLIT == 1) {
          st_sc1(&part[(j - J0) * BM + (i - I0)], acc[tj][ti][r]);
        } else if (i < a.ni && j < a.nj && (!a.tri || i >= j)) {
          double* cp = a.C + j * a.ldc + i;
          if (cinit) {
            double v = acc[tj][ti][r];
            if (SPLIT == 2) v += ld_sc1(&part[(j - J0) * BM + (i - I0)]);
            if (SC1OUT) st_sc1(cp, v);
            else *cp = v;
          } else {
            double av = acc[tj][ti][r];
            if (SPLITADD && SPLIT == 2) av += ld_sc1(&part[(j - J0) * BM + (i - I0)]);
            double v = a.alpha * av;
            if (a.beta != 0.0) v += a.beta * (PRE ? pc[ti][r] : *cp);
            if (a.P) v += a.tP * (PRE ? pp[ti][r] : a.P[j * a.ldp + i]);
            if (a.dvec && i == j) v += a.dvec[i];
            *cp = v;
          }
        }
      }
    }
  }
  if (SPLIT == 1) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (tid == 0) __hip_atomic_store(pflag, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (SPLIT == 2) {
    // the partial is consumed (its loads fed the stores above): the flag goes back to zero
    __syncthreads();
    if (tid == 0) __hip_atomic_store(pflag, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
#ifdef IPM_TILE_STAMPS
  IPM_TSTAMP(3);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  IPM_TSTAMP(4);
  IPM_TSTAMPR(7);
#endif
}

// the tile mfma_tile would take for index Lw (same enumeration), and whether it is full with whole
// 16-row K slabs (no split pieces: callers of the fast loop)
template <int BM>
__device__ __forceinline__ bool tile_fast_ok(const GemmArgs& a, int64_t Lw) {
  int64_t L = Lw, bi, bj;
  const int64_t q = a.nblk >> 3;
  if (a.xcd_remap && !a.rowmajor && L < (q << 3)) L = (L & 7) * q + (L >> 3);
  if (a.rowmajor) {
    bi = L / a.tiles_j;
    bj = L % a.tiles_j;
  } else if (a.tri) {
    int64_t b = (int64_t)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while ((b + 1) * (b + 2) / 2 <= L) ++b;
    while (b * (b + 1) / 2 > L) --b;
    bi = b;
    bj = L - b * (b + 1) / 2;
  } else {
    bi = L % a.tiles_i;
    bj = L / a.tiles_i;
  }
  return (bi + 1) * BM <= a.ni && (bj + 1) * BM <= a.nj && (a.K % 16) == 0;
}

// the fast loop of the GEMM / SYRK kernels: 2 (X fragments from memory, Y through LDS; r6), 1 (both
// through LDS), 3 (both from memory)
#ifndef IPM_SYRK_LOOP
#define IPM_SYRK_LOOP 2
#endif

template <int BM_, bool WEIGHT, bool VEC, int WJ = 2>
__global__ __launch_bounds__(128 * WJ, 2 / (WJ / 2)) void k_mfma_gemm(GemmArgs a) {
  if (a.info && *a.info != 0) return;
  __shared__ MfSmem<BM_, WJ> sm;
  for (int64_t Lw = blockIdx.x; Lw < a.nblk; Lw += gridDim.x) {
    if (BM_ == 128 && VEC && WJ == 2 && tile_fast_ok<BM_>(a, Lw))
      mfma_tile<BM_, WEIGHT, VEC, WJ, false, false, (BM_ == 128 && VEC && WJ == 2) ? IPM_SYRK_LOOP : 0>(a, Lw, sm);
    else
      mfma_tile<BM_, WEIGHT, VEC, WJ>(a, Lw, sm);
  }
}

// Split tail (the KKT SYRK): blocks [0, s_full) run whole tiles; then each of the last q tiles of
// the enumeration as two K halves, the upper half first (lower blockIdx; blocks are dispatched in
// order, so the half that waits always has its partner resident or done) -> partial tile in
// sscr + p * BM * BM, flag sflag[p] (zeroed before the launch).  The last round of a
// lower-triangle grid (e.g. 2080 tiles on 512 slots: a fifth round of 32) then runs as half
// tiles on twice the slots.  The sum order (lower half, + upper half) is fixed: deterministic.
template <int BM_, bool WEIGHT, bool VEC>
__global__ __launch_bounds__(256, 2) void k_mfma_gemm_split(GemmArgs a, int64_t s_full, double* sscr,
                                                            unsigned* sflag) {
  if (a.info && *a.info != 0) return;
  __shared__ MfSmem<BM_, 2> sm;
  const int64_t b = blockIdx.x;
  constexpr int FL = (BM_ == 128 && VEC) ? IPM_SYRK_LOOP : 0;
  if (b < s_full) {
    if (FL && tile_fast_ok<BM_>(a, b)) mfma_tile<BM_, WEIGHT, VEC, 2, false, true, FL>(a, b, sm);
    else mfma_tile<BM_, WEIGHT, VEC, 2, false, true>(a, b, sm);
    return;
  }
  const int64_t u = b - s_full, p = u >> 1;
  double* part = sscr + p * (int64_t)(BM_ * BM_);
  const int64_t Lw = s_full + p;
  if (FL && (a.K % 32) == 0 && tile_fast_ok<BM_>(a, Lw))
    mfma_tile<BM_, WEIGHT, VEC, 2, false, true, FL>(a, Lw, sm, (u & 1) ? 2 : 1, part, sflag + p);
  else
    mfma_tile<BM_, WEIGHT, VEC, 2, false, true>(a, Lw, sm, (u & 1) ? 2 : 1, part, sflag + p);
}

// Stream-K tail (the KKT SYRK on 128-tiles): a lower-triangle grid of nt = R * slots + q tiles
// runs R whole rounds, and its last q tiles as P K pieces each (q * P <= slots), so that the
// partial last round becomes one short round of pieces on (nearly) every slot instead of q whole
// tiles on q slots (2080 tiles on 512 slots: 4 rounds + 512 pieces of K/16).  Blocks [0, npc)
// are the pieces, dispatched FIRST: piece u = tile s_full + u / P, K range [p Kp, min(K, p Kp +
// Kp)), p = u % P; its partial goes to sscr + u * BM * BM (sc1).  The piece that arrives last at
// the tile's counter (cnt[u / P], zeroed before the launch) sums the P partials in the fixed
// order p = 0 .. P-1 and applies the epilogue: deterministic, and nobody waits.  Blocks
// [npc, npc + s_full) are the whole tiles.
template <int BM>
__device__ __forceinline__ void tile_ij(const GemmArgs& a, int64_t Lw, int64_t& bi, int64_t& bj) {
  int64_t L = Lw;
  const int64_t q = a.nblk >> 3;
  if (a.xcd_remap && !a.rowmajor && L < (q << 3)) L = (L & 7) * q + (L >> 3);
  if (a.rowmajor) {
    bi = L / a.tiles_j;
    bj = L % a.tiles_j;
  } else if (a.tri) {
    int64_t b = (int64_t)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while ((b + 1) * (b + 2) / 2 <= L) ++b;
    while (b * (b + 1) / 2 > L) --b;
    bi = b;
    bj = L - b * (b + 1) / 2;
  } else {
    bi = L % a.tiles_i;
    bj = L / a.tiles_i;
  }
}

template <bool WEIGHT, bool VEC>
__global__ __launch_bounds__(256, 2) void k_mfma_gemm_streamk(GemmArgs a, int64_t s_full, int P, int64_t Kp,
                                                              int64_t npc, double* sscr, unsigned* cnt,
                                                              int pieces_last) {
  constexpr int BM = 128;
  if (a.info && *a.info != 0) return;
  __shared__ MfSmem<BM, 2> sm;
  __shared__ int slast;
  int64_t b = blockIdx.x;
  constexpr int FL = VEC ? IPM_SYRK_LOOP : 0;
  // block order: pieces first (default) or whole tiles first
  bool whole;
  if (pieces_last) {
    whole = b < s_full;
    if (!whole) b -= s_full;
  } else {
    whole = b >= npc;
  }
  if (whole) {
    const int64_t L = pieces_last ? b : b - npc;
    if (FL && tile_fast_ok<BM>(a, L)) mfma_tile<BM, WEIGHT, VEC, 2, false, true, FL>(a, L, sm);
    else mfma_tile<BM, WEIGHT, VEC, 2, false, true>(a, L, sm);
    return;
  }
  const int64_t ti = b / P, p = b - ti * P, L = s_full + ti;
  const int64_t k0 = p * Kp, k1 = std::min<int64_t>(a.K, k0 + Kp);
  double* part = sscr + b * (int64_t)(BM * BM);
  // (the flag mfma_tile raises after its partial: a per-piece word past the tile counters)
  unsigned* pf = cnt + (a.nblk - s_full) + b;
  if (FL && (k0 % 16) == 0 && ((k1 - k0) % 16) == 0 && tile_fast_ok<BM>(a, L))
    mfma_tile<BM, WEIGHT, VEC, 2, false, true, FL>(a, L, sm, 1, part, pf, k0, k1);
  else
    mfma_tile<BM, WEIGHT, VEC, 2, false, true>(a, L, sm, 1, part, pf, k0, k1);
  // (mfma_tile ended with s_waitcnt vmcnt(0) + barrier after the partial's sc1 stores)
  const int tid = threadIdx.x;
  if (tid == 0)
    slast = __hip_atomic_fetch_add(&cnt[ti], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(P - 1);
  __syncthreads();
  if (!slast) return;
  int64_t bi, bj;
  tile_ij<BM>(a, L, bi, bj);
  const int64_t I0 = bi * BM, J0 = bj * BM;
  const bool cinit = a.sub || a.accum || (a.beta == 1.0 && a.alpha == -1.0 && !a.P && !a.dvec);
  const double* base = sscr + ti * P * (int64_t)(BM * BM);
  // column-major tile: consecutive threads take consecutive i (coalesced partial and C traffic).
  // 4 elements per pass (8 with 4 pieces) with all their partial loads issued back to back (the partials come
  // from other CUs' stores: a memory round trip each), then the fixed-order sums p = 0 .. P-1.  The
  // piece count is a compile-time constant in the common plans (4 / 8 / 16): with a run-time bound
  // every load sat in its own conditional block and the compiler waited for each one -- the fixup
  // of a 16-piece tile took ~200 us (r6, tools/syrk_lab.hip).
  auto fixup = [&](auto pc) {
    constexpr int NP = decltype(pc)::value, U = NP >= 8 ? 4 : 8;
    for (int e0 = tid; e0 < BM * BM; e0 += U * 256) {
      // every load of the pass (the partials, and the P / C values the epilogue reads) before its
      // first store: vmcnt counts loads and stores in issue order, so a load behind a store waits
      // for the store too -- one element at a time, the fixup was store-latency-bound
      double pv[U][NP], pp[U], cv[U];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int q = 0; q < NP; ++q) pv[u][q] = ld_sc1(&base[q * (int64_t)(BM * BM) + e0 + 256 * u]);
      bool ok[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int e = e0 + 256 * u;
        const int64_t i = I0 + (e & (BM - 1)), j = J0 + e / BM;
        ok[u] = !(i >= a.ni || j >= a.nj || (a.tri && i < j));
        pp[u] = (ok[u] && !cinit && a.P) ? a.P[j * a.ldp + i] : 0.0;
        cv[u] = (ok[u] && (cinit || a.beta != 0.0)) ? a.C[j * a.ldc + i] : 0.0;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (!ok[u]) continue;
        const int e = e0 + 256 * u;
        const int64_t i = I0 + (e & (BM - 1)), j = J0 + e / BM;
        double sum = 0.0;
#pragma unroll
        for (int q = 0; q < NP; ++q) sum += pv[u][q];
        double* cp = a.C + j * a.ldc + i;
        if (cinit) {
          *cp = cv[u] + sum;
        } else {
          double v = a.alpha * sum;
          if (a.beta != 0.0) v += a.beta * cv[u];
          if (a.P) v += a.tP * pp[u];
          if (a.dvec && i == j) v += a.dvec[i];
          *cp = v;
        }
      }
    }
  };
  if (P == 16) fixup(std::integral_constant<int, 16>{});
  else if (P == 8) fixup(std::integral_constant<int, 8>{});
  else if (P == 4) fixup(std::integral_constant<int, 4>{});
  else {
    for (int e = tid; e < BM * BM; e += 256) {
      const int il = e & (BM - 1), jl = e / BM;
      const int64_t i = I0 + il, j = J0 + jl;
      if (i >= a.ni || j >= a.nj || (a.tri && i < j)) continue;
      double pv[16];
#pragma unroll
      for (int q = 0; q < 16; ++q) pv[q] = q < P ? ld_sc1(&base[q * (int64_t)(BM * BM) + e]) : 0.0;
      double sum = 0.0;
#pragma unroll
      for (int q = 0; q < 16; ++q)
        if (q < P) sum += pv[q];
      double* cp = a.C + j * a.ldc + i;
      if (cinit) {
        *cp = *cp + sum;
      } else {
        double v = a.alpha * sum;
        if (a.beta != 0.0) v += a.beta * (*cp);
        if (a.P) v += a.tP * a.P[j * a.ldp + i];
        if (a.dvec && i == j) v += a.dvec[i];
        *cp = v;
      }
    }
  }
  IPM_TSTAMPR(7);   // (lab stamps: the fixup's end replaces the piece's exit)
  // every piece of this tile has counted: the counter goes back to zero for the next launch
  if (tid == 0) __hip_atomic_store(&cnt[ti], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// stream-K plan for nt 128-tiles on `slots` slots: pieces per tile P (0: not worth it) and the
// piece length Kp (whole 16-row slabs); the last piece of a tile may be shorter
// IPM_STREAMK: 0 off (the K-halves split tail), 1 pieces first, 2 pieces last (the default), 3
// pieces first with at most 8 pieces per tile, 4 pieces last with at most 8.  Rounds 2-5 defaulted
// to 3 from two rounds of tiles up (2.37 -> 2.30 ms at n = 8192, K = 2048; profiles/r2_streamk_ab.txt)
// and to 2 below (SOCP n = 4096, 528 tiles on 512 slots: 1.51 -> 1.46 ms, profiles/r4q); with the
// r6 tile loop and fixup, 2 is ahead at n = 8192 too (bench A/B: 2.200 vs 2.220 ms,
// profiles/r6_syrk_lab/bench_ab_streamk.txt)
inline int streamk_mode(int64_t nt = 0, int slots = 0) {
  static const int env = [] {
    const char* e = getenv("IPM_STREAMK");
    return e ? atoi(e) : -1;
  }();
  if (env >= 0) return env;
  (void)nt;
  (void)slots;
  return 2;
}
inline int streamk_plan(int64_t nt, int slots, int64_t cap, int64_t K, int64_t& q, int64_t& Kp) {
  const int mode = streamk_mode(nt, slots);
  q = 0;
  Kp = 0;
  if (!mode || slots <= 0 || nt < slots) return 0;
  q = nt % slots;
  if (q == 0) return 0;
  const int pmax = (mode == 3 || mode == 4) ? 8 : 16;
  int P = 1;
  while (P * 2 <= pmax && q * P * 2 <= slots && q * P * 2 <= cap && K / (P * 2) >= 64) P *= 2;
  if (P < 4) return 0;
  Kp = ((K + P - 1) / P + 15) / 16 * 16;
  P = (int)((K + Kp - 1) / Kp);
  return P >= 4 ? P : 0;
}

// how many of nt tiles to split: list schedule on `slots` workgroup slots (2 per CU), whole tile
// 1.0, half tile 0.55; the q with the smallest makespan (cached per grid)
inline int64_t gemm_split_plan(int64_t nt, int slots, int64_t cap) {
  if (nt <= 0 || slots <= 0) return 0;
  static std::mutex mu;
  static std::map<std::tuple<int64_t, int, int64_t>, int64_t> cache;
  std::lock_guard<std::mutex> lk(mu);
  const auto key = std::make_tuple(nt, slots, cap);
  auto it = cache.find(key);
  if (it != cache.end()) return it->second;
  auto mk = [&](int64_t q) {
    std::priority_queue<double, std::vector<double>, std::greater<double>> pq;
    for (int i = 0; i < slots; ++i) pq.push(0.0);
    double m = 0.0;
    auto put = [&](double d) {
      const double t = pq.top() + d;
      pq.pop();
      pq.push(t);
      m = std::max(m, t);
    };
    for (int64_t i = 0; i < nt - q; ++i) put(1.0);
    for (int64_t i = 0; i < 2 * q; ++i) put(0.55);
    return m;
  };
  double best = mk(0);
  int64_t bq = 0;
  for (int64_t q = 8; q <= std::min(nt, cap); q += 8) {
    const double m = mk(q);
    if (m < best - 0.02) {
      best = m;
      bq = q;
    }
  }
  cache[key] = bq;
  return bq;
}

template <int BM>
inline void mfma_gemm_launch_bm(hipStream_t st, GemmArgs a, bool vec) {
  const int64_t ti = (a.ni + BM - 1) / BM, tj = (a.nj + BM - 1) / BM;
  a.tiles_i = ti;
  a.nblk = a.tri ? ti * (ti + 1) / 2 : ti * tj;
  dim3 g((unsigned)a.nblk), b(256);
  if (a.w) {
    if (vec) hipLaunchKernelGGL((k_mfma_gemm<BM, true, true>), g, b, 0, st, a);
    else hipLaunchKernelGGL((k_mfma_gemm<BM, true, false>), g, b, 0, st, a);
  } else {
    if (vec) hipLaunchKernelGGL((k_mfma_gemm<BM, false, true>), g, b, 0, st, a);
    else hipLaunchKernelGGL((k_mfma_gemm<BM, false, false>), g, b, 0, st, a);
  }
}

// launch helper: picks the tile size (grid fill), the weighted / vector-load instantiation
inline void mfma_gemm_launch(hipStream_t st, GemmArgs a) {
  if (a.ni <= 0 || a.nj <= 0) return;
  const bool vec = ((a.ldx & 1) == 0) && ((a.ldy & 1) == 0) && ((((uintptr_t)a.X) & 15) == 0) &&
                   ((((uintptr_t)a.Y) & 15) == 0);
  const int64_t ti = (a.ni + 127) / 128, tj = (a.nj + 127) / 128;
  const int64_t nblk128 = a.tri ? ti * (ti + 1) / 2 : ti * tj;
  if (nblk128 >= 768) mfma_gemm_launch_bm<128>(st, a, vec);
  else mfma_gemm_launch_bm<64>(st, a, vec);
}

// the KKT SYRK with its tail split (ws: cap * BM * BM doubles of partial tiles, then cap flags);
// falls back to the plain launch when nothing is worth splitting
inline void mfma_gemm_launch_split(hipStream_t st, GemmArgs a, double* ws, int64_t cap, int slots,
                                   bool flags_zero = false) {
  if (a.ni <= 0 || a.nj <= 0) return;
  const bool vec = ((a.ldx & 1) == 0) && ((a.ldy & 1) == 0) && ((((uintptr_t)a.X) & 15) == 0) &&
                   ((((uintptr_t)a.Y) & 15) == 0);
  const int64_t ti128 = (a.ni + 127) / 128, tj128 = (a.nj + 127) / 128;
  const int64_t nblk128 = a.tri ? ti128 * (ti128 + 1) / 2 : ti128 * tj128;
  int BM = nblk128 >= 768 ? 128 : 64;
  if (BM == 64 && ws) {
    // a 128-tile grid just past whole rounds of the slots (SOCP n = 4096: 528 tiles on 512) takes
    // the stream-K tail too, instead of the 64-tile grid's half-rate tiles
    int64_t q0 = 0, K0 = 0;
    if (streamk_plan(nblk128, slots, cap, a.K, q0, K0) > 0) BM = 128;
  }
  const int64_t ti = (a.ni + BM - 1) / BM, tj = (a.nj + BM - 1) / BM;
  a.tiles_i = ti;
  a.nblk = a.tri ? ti * (ti + 1) / 2 : ti * tj;
  if (BM == 128 && ws) {
    int64_t qk = 0, Kp = 0;
    const int P = streamk_plan(a.nblk, slots, cap, a.K, qk, Kp);
    if (P > 0) {
      const int64_t s_full = a.nblk - qk, npc = qk * P;
      // counters: qk tile words, then npc per-piece words (ws has cap * 128 * 128 doubles of
      // partials, then the flag area)
      unsigned* cnt = reinterpret_cast<unsigned*>(ws + cap * (int64_t)(128 * 128));
      if (!flags_zero) hipMemsetAsync(cnt, 0, qk * sizeof(unsigned), st);   // (per-piece words: never waited on)
      dim3 g((unsigned)(npc + s_full)), blk(256);
      const int pl = (streamk_mode(a.nblk, slots) == 2 || streamk_mode(a.nblk, slots) == 4) ? 1 : 0;
      if (a.w) {
        if (vec) hipLaunchKernelGGL((k_mfma_gemm_streamk<true, true>), g, blk, 0, st, a, s_full, P, Kp, npc, ws, cnt, pl);
        else hipLaunchKernelGGL((k_mfma_gemm_streamk<true, false>), g, blk, 0, st, a, s_full, P, Kp, npc, ws, cnt, pl);
      } else {
        if (vec) hipLaunchKernelGGL((k_mfma_gemm_streamk<false, true>), g, blk, 0, st, a, s_full, P, Kp, npc, ws, cnt, pl);
        else hipLaunchKernelGGL((k_mfma_gemm_streamk<false, false>), g, blk, 0, st, a, s_full, P, Kp, npc, ws, cnt, pl);
      }
      return;
    }
  }
  // (the K-halves planner keeps its round-2 cap of 256 tiles)
  const int64_t q = ws ? gemm_split_plan(a.nblk, slots, std::min<int64_t>(cap, 256)) : 0;
  if (q == 0) {
    if (BM == 128) mfma_gemm_launch_bm<128>(st, a, vec);
    else mfma_gemm_launch_bm<64>(st, a, vec);
    return;
  }
  const int64_t s_full = a.nblk - q;
  unsigned* flags = reinterpret_cast<unsigned*>(ws + cap * (int64_t)(128 * 128));
  if (!flags_zero) hipMemsetAsync(flags, 0, q * sizeof(unsigned), st);
  dim3 g((unsigned)(s_full + 2 * q)), b(256);
#define IPM_SPLIT_LAUNCH(BMv)                                                                             \
  do {                                                                                                    \
    if (a.w) {                                                                                            \
      if (vec) hipLaunchKernelGGL((k_mfma_gemm_split<BMv, true, true>), g, b, 0, st, a, s_full, ws, flags);   \
      else hipLaunchKernelGGL((k_mfma_gemm_split<BMv, true, false>), g, b, 0, st, a, s_full, ws, flags);      \
    } else {                                                                                              \
      if (vec) hipLaunchKernelGGL((k_mfma_gemm_split<BMv, false, true>), g, b, 0, st, a, s_full, ws, flags);  \
      else hipLaunchKernelGGL((k_mfma_gemm_split<BMv, false, false>), g, b, 0, st, a, s_full, ws, flags);     \
    }                                                                                                     \
  } while (0)
  if (BM == 128) IPM_SPLIT_LAUNCH(128);
  else IPM_SPLIT_LAUNCH(64);
#undef IPM_SPLIT_LAUNCH
}

}  // namespace ipm
