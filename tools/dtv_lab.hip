// fp64 MFMA tile-loop lab (diagnostic only): C = X^T diag(w) Y on k-major operands, full square grid
// of 128 x 128 tiles, 256 threads, BK = 16 -- the library's fast loop (ipm_mfma.h mfma_tile LOOP 1)
// against
//   V1: X fragments loaded from global memory straight into the MFMA operand registers (only Y is
//       staged through LDS); each k-row's X fragment is reloaded for the next slab right after its
//       MFMAs (one slab of prefetch, no extra registers)
//   V2: both operands through LDS, the next k-step's fragments read before this k-step's MFMAs
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/dtv_lab.hip -o build/r6lab/dtv_lab
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../interiorpoint-gpu_amd/csrc/ipm_mfma.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

typedef double dbl4 __attribute__((ext_vector_type(4)));
constexpr int BM = 128, BK = 16, LD = BM + 16, PT = 8, TPR = 16, TW = 4;

__global__ __launch_bounds__(256, 2) void k_v0(ipm::GemmArgs a) {
  __shared__ ipm::MfSmem<128, 2> sm;
  ipm::mfma_tile<128, true, true, 2, false, false, 1>(a, blockIdx.x, sm);
}

// epilogue shared by the variants: C(i, j) = acc, column-major C
__device__ __forceinline__ void store_tile(const ipm::GemmArgs& a, int64_t I0, int64_t J0, int wi, int wj, int fr,
                                           int fk, dbl4 (&acc)[TW][TW]) {
#pragma unroll
  for (int tj = 0; tj < TW; ++tj)
#pragma unroll
    for (int ti = 0; ti < TW; ++ti) {
      const int64_t i = I0 + wi * 64 + ti * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int64_t j = J0 + wj * 64 + tj * 16 + fk + 4 * r;
        a.C[j * a.ldc + i] = acc[tj][ti][r];
      }
    }
}

template <bool WEIGHT>
__global__ __launch_bounds__(256, 2) void k_v1(ipm::GemmArgs a) {
  __shared__ alignas(16) double sY[2][BK * LD];
  const int64_t L = blockIdx.x, bi = L % a.tiles_i, bj = L / a.tiles_i;
  const int64_t I0 = bi * BM, J0 = bj * BM;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wi = wv & 1, wj = wv >> 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int sr = tid / TPR, sc = (tid % TPR) * PT;
  const int64_t nslab = a.K / BK;
  const double* yp = a.Y + sr * a.ldy + J0 + sc;
  // this lane's X fragment elements: X[k = s*16 + kk*4 + fk][I0 + wi*64 + t*16 + fr]
  const double* xq = a.X + (int64_t)fk * a.ldx + I0 + wi * 64 + fr;
  const double* wq = a.w + fk;
  double fy[PT];
  auto fload = [&](int64_t s) {
    const double2* ys = reinterpret_cast<const double2*>(yp + s * BK * a.ldy);
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
  double xr[4][TW], wk[4];
  auto xload = [&](int64_t s, int kk) {
    const double* p = xq + (s * BK + kk * 4) * a.ldx;
#pragma unroll
    for (int t = 0; t < TW; ++t) xr[kk][t] = p[t * 16];
    if (WEIGHT) wk[kk] = wq[s * BK + kk * 4];
  };
  dbl4 acc[TW][TW];
#pragma unroll
  for (int u = 0; u < TW; ++u)
#pragma unroll
    for (int v = 0; v < TW; ++v) acc[u][v] = dbl4{0.0, 0.0, 0.0, 0.0};
  fload(0);
  fstore(0);
  fload(nslab > 1 ? 1 : 0);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) xload(0, kk);
  __syncthreads();
  for (int64_t s = 0; s < nslab; ++s) {
    const int buf = (int)(s & 1);
    const double* by = sY[buf];
    fstore(buf ^ 1);
    fload(std::min<int64_t>(s + 2, nslab - 1));
    const int64_t sn = std::min<int64_t>(s + 1, nslab - 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      double av[TW], bv[TW];
#pragma unroll
      for (int t = 0; t < TW; ++t) av[t] = by[(kk * 4 + fk) * LD + wj * 64 + t * 16 + fr];
#pragma unroll
      for (int t = 0; t < TW; ++t) bv[t] = WEIGHT ? xr[kk][t] * wk[kk] : xr[kk][t];
      xload(sn, kk);
#pragma unroll
      for (int tj = 0; tj < TW; ++tj)
#pragma unroll
        for (int ti = 0; ti < TW; ++ti)
          acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tj], bv[ti], acc[tj][ti], 0, 0, 0);
    }
    __syncthreads();
  }
  store_tile(a, I0, J0, wi, wj, fr, fk, acc);
}

template <bool WEIGHT>
__global__ __launch_bounds__(256, 2) void k_v2(ipm::GemmArgs a) {
  __shared__ alignas(16) double sX[2][BK * LD];
  __shared__ alignas(16) double sY[2][BK * LD];
  const int64_t L = blockIdx.x, bi = L % a.tiles_i, bj = L / a.tiles_i;
  const int64_t I0 = bi * BM, J0 = bj * BM;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wi = wv & 1, wj = wv >> 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int sr = tid / TPR, sc = (tid % TPR) * PT;
  const int64_t nslab = a.K / BK;
  const double* xp = a.X + sr * a.ldx + I0 + sc;
  const double* yp = a.Y + sr * a.ldy + J0 + sc;
  double fx[PT], fy[PT], fw = 1.0;
  auto fload = [&](int64_t s) {
    const double2* xs = reinterpret_cast<const double2*>(xp + s * BK * a.ldx);
    const double2* ys = reinterpret_cast<const double2*>(yp + s * BK * a.ldy);
#pragma unroll
    for (int q = 0; q < PT / 2; ++q) {
      const double2 u = xs[q], v = ys[q];
      fx[2 * q] = u.x; fx[2 * q + 1] = u.y;
      fy[2 * q] = v.x; fy[2 * q + 1] = v.y;
    }
    if (WEIGHT) fw = a.w[s * BK + sr];
  };
  auto fstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < PT; ++q) {
      sX[buf][sr * LD + sc + q] = WEIGHT ? fx[q] * fw : fx[q];
      sY[buf][sr * LD + sc + q] = fy[q];
    }
  };
  dbl4 acc[TW][TW];
#pragma unroll
  for (int u = 0; u < TW; ++u)
#pragma unroll
    for (int v = 0; v < TW; ++v) acc[u][v] = dbl4{0.0, 0.0, 0.0, 0.0};
  fload(0);
  fstore(0);
  fload(nslab > 1 ? 1 : 0);
  __syncthreads();
  double av[2][TW], bv[2][TW];
  auto fragload = [&](const double* bx, const double* by, int kk, int p) {
#pragma unroll
    for (int t = 0; t < TW; ++t) av[p][t] = by[(kk * 4 + fk) * LD + wj * 64 + t * 16 + fr];
#pragma unroll
    for (int t = 0; t < TW; ++t) bv[p][t] = bx[(kk * 4 + fk) * LD + wi * 64 + t * 16 + fr];
  };
  fragload(sX[0], sY[0], 0, 0);
  for (int64_t s = 0; s < nslab; ++s) {
    const int buf = (int)(s & 1);
    fstore(buf ^ 1);
    fload(std::min<int64_t>(s + 2, nslab - 1));
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk < 3) fragload(sX[buf], sY[buf], kk + 1, (kk + 1) & 1);
#pragma unroll
      for (int tj = 0; tj < TW; ++tj)
#pragma unroll
        for (int ti = 0; ti < TW; ++ti)
          acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kk & 1][tj], bv[kk & 1][ti], acc[tj][ti], 0, 0, 0);
    }
    __syncthreads();
    fragload(sX[buf ^ 1], sY[buf ^ 1], 0, 0);
  }
  store_tile(a, I0, J0, wi, wj, fr, fk, acc);
}

// V3: both operands straight to registers, no LDS, no barriers
template <bool WEIGHT>
__global__ __launch_bounds__(256, 2) void k_v3(ipm::GemmArgs a) {
  const int64_t L = blockIdx.x, bi = L % a.tiles_i, bj = L / a.tiles_i;
  const int64_t I0 = bi * BM, J0 = bj * BM;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wi = wv & 1, wj = wv >> 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int64_t nslab = a.K / BK;
  const double* xq = a.X + (int64_t)fk * a.ldx + I0 + wi * 64 + fr;
  const double* yq = a.Y + (int64_t)fk * a.ldy + J0 + wj * 64 + fr;
  const double* wq = a.w + fk;
  double xr[4][TW], yr[4][TW], wk[4];
  auto load = [&](int64_t s, int kk) {
    const double* p = xq + (s * BK + kk * 4) * a.ldx;
    const double* q = yq + (s * BK + kk * 4) * a.ldy;
#pragma unroll
    for (int t = 0; t < TW; ++t) xr[kk][t] = p[t * 16];
#pragma unroll
    for (int t = 0; t < TW; ++t) yr[kk][t] = q[t * 16];
    if (WEIGHT) wk[kk] = wq[s * BK + kk * 4];
  };
  dbl4 acc[TW][TW];
#pragma unroll
  for (int u = 0; u < TW; ++u)
#pragma unroll
    for (int v = 0; v < TW; ++v) acc[u][v] = dbl4{0.0, 0.0, 0.0, 0.0};
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) load(0, kk);
  for (int64_t s = 0; s < nslab; ++s) {
    const int64_t sn = std::min<int64_t>(s + 1, nslab - 1);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      double av[TW], bv[TW];
#pragma unroll
      for (int t = 0; t < TW; ++t) av[t] = yr[kk][t];
#pragma unroll
      for (int t = 0; t < TW; ++t) bv[t] = WEIGHT ? xr[kk][t] * wk[kk] : xr[kk][t];
      load(sn, kk);
#pragma unroll
      for (int tj = 0; tj < TW; ++tj)
#pragma unroll
        for (int ti = 0; ti < TW; ++ti)
          acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tj], bv[ti], acc[tj][ti], 0, 0, 0);
    }
  }
  store_tile(a, I0, J0, wi, wj, fr, fk, acc);
}

// V4: V1 with two slabs of X prefetch (the reload of slab s+2 after the k-row's MFMAs)
template <bool WEIGHT>
__global__ __launch_bounds__(256, 2) void k_v4(ipm::GemmArgs a) {
  __shared__ alignas(16) double sY[2][BK * LD];
  const int64_t L = blockIdx.x, bi = L % a.tiles_i, bj = L / a.tiles_i;
  const int64_t I0 = bi * BM, J0 = bj * BM;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wi = wv & 1, wj = wv >> 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int sr = tid / TPR, sc = (tid % TPR) * PT;
  const int64_t nslab = a.K / BK;
  const double* yp = a.Y + sr * a.ldy + J0 + sc;
  const double* xq = a.X + (int64_t)fk * a.ldx + I0 + wi * 64 + fr;
  const double* wq = a.w + fk;
  double fy[PT];
  auto fload = [&](int64_t s) {
    const double2* ys = reinterpret_cast<const double2*>(yp + s * BK * a.ldy);
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
  double xr[2][4][TW], wk[2][4];
  auto xload = [&](int64_t s, int kk, int p) {
    const double* q = xq + (s * BK + kk * 4) * a.ldx;
#pragma unroll
    for (int t = 0; t < TW; ++t) xr[p][kk][t] = q[t * 16];
    if (WEIGHT) wk[p][kk] = wq[s * BK + kk * 4];
  };
  dbl4 acc[TW][TW];
#pragma unroll
  for (int u = 0; u < TW; ++u)
#pragma unroll
    for (int v = 0; v < TW; ++v) acc[u][v] = dbl4{0.0, 0.0, 0.0, 0.0};
  fload(0);
  fstore(0);
  fload(nslab > 1 ? 1 : 0);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) xload(0, kk, 0);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) xload(nslab > 1 ? 1 : 0, kk, 1);
  __syncthreads();
  // slabs in pairs (register set p = s & 1 without dynamic indexing); nslab even
  for (int64_t s = 0; s < nslab; s += 2) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int64_t sc_ = s + h;
      const int buf = h;
      const double* by = sY[buf];
      fstore(buf ^ 1);
      fload(std::min<int64_t>(sc_ + 2, nslab - 1));
      const int64_t sn = std::min<int64_t>(sc_ + 2, nslab - 1);
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        double av[TW], bv[TW];
#pragma unroll
        for (int t = 0; t < TW; ++t) av[t] = by[(kk * 4 + fk) * LD + wj * 64 + t * 16 + fr];
#pragma unroll
        for (int t = 0; t < TW; ++t) bv[t] = WEIGHT ? xr[h][kk][t] * wk[h][kk] : xr[h][kk][t];
        xload(sn, kk, h);
#pragma unroll
        for (int tj = 0; tj < TW; ++tj)
#pragma unroll
          for (int ti = 0; ti < TW; ++ti)
            acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tj], bv[ti], acc[tj][ti], 0, 0, 0);
      }
      __syncthreads();
    }
  }
  store_tile(a, I0, J0, wi, wj, fr, fk, acc);
}

// V6: V1 with the Y fragments of k-step kk + 1 read from LDS before k-step kk's MFMAs
template <bool WEIGHT>
__global__ __launch_bounds__(256, 2) void k_v6(ipm::GemmArgs a) {
  __shared__ alignas(16) double sY[2][BK * LD];
  const int64_t L = blockIdx.x, bi = L % a.tiles_i, bj = L / a.tiles_i;
  const int64_t I0 = bi * BM, J0 = bj * BM;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wi = wv & 1, wj = wv >> 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int sr = tid / TPR, sc = (tid % TPR) * PT;
  const int64_t nslab = a.K / BK;
  const double* yp = a.Y + sr * a.ldy + J0 + sc;
  const double* xq = a.X + (int64_t)fk * a.ldx + I0 + wi * 64 + fr;
  const double* wq = a.w + fk;
  double fy[PT];
  auto fload = [&](int64_t s) {
    const double2* ys = reinterpret_cast<const double2*>(yp + s * BK * a.ldy);
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
  double xr[4][TW], wk[4];
  auto xload = [&](int64_t s, int kk) {
    const double* p = xq + (s * BK + kk * 4) * a.ldx;
#pragma unroll
    for (int t = 0; t < TW; ++t) xr[kk][t] = p[t * 16];
    if (WEIGHT) wk[kk] = wq[s * BK + kk * 4];
  };
  dbl4 acc[TW][TW];
#pragma unroll
  for (int u = 0; u < TW; ++u)
#pragma unroll
    for (int v = 0; v < TW; ++v) acc[u][v] = dbl4{0.0, 0.0, 0.0, 0.0};
  fload(0);
  fstore(0);
  fload(nslab > 1 ? 1 : 0);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) xload(0, kk);
  __syncthreads();
  double av[2][TW];
#pragma unroll
  for (int t = 0; t < TW; ++t) av[0][t] = sY[0][fk * LD + wj * 64 + t * 16 + fr];
  for (int64_t s = 0; s < nslab; ++s) {
    const int buf = (int)(s & 1);
    const double* by = sY[buf];
    fstore(buf ^ 1);
    fload(std::min<int64_t>(s + 2, nslab - 1));
    const int64_t sn = std::min<int64_t>(s + 1, nslab - 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < 4; ++kk) {
      if (kk < 3) {
#pragma unroll
        for (int t = 0; t < TW; ++t) av[(kk + 1) & 1][t] = by[((kk + 1) * 4 + fk) * LD + wj * 64 + t * 16 + fr];
      }
      double bv[TW];
#pragma unroll
      for (int t = 0; t < TW; ++t) bv[t] = WEIGHT ? xr[kk][t] * wk[kk] : xr[kk][t];
      xload(sn, kk);
#pragma unroll
      for (int tj = 0; tj < TW; ++tj)
#pragma unroll
        for (int ti = 0; ti < TW; ++ti)
          acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[kk & 1][tj], bv[ti], acc[tj][ti], 0, 0, 0);
    }
    __syncthreads();
#pragma unroll
    for (int t = 0; t < TW; ++t) av[0][t] = sY[buf ^ 1][fk * LD + wj * 64 + t * 16 + fr];
  }
  store_tile(a, I0, J0, wi, wj, fr, fk, acc);
}

// V7: V1 with two slabs per barrier (four LDS buffers of Y: the stores of slabs s+2, s+3 and the
// loads of s+4, s+5 once per pair)
template <bool WEIGHT>
__global__ __launch_bounds__(256, 2) void k_v7(ipm::GemmArgs a) {
  __shared__ alignas(16) double sY[4][BK * LD];
  const int64_t L = blockIdx.x, bi = L % a.tiles_i, bj = L / a.tiles_i;
  const int64_t I0 = bi * BM, J0 = bj * BM;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6, wi = wv & 1, wj = wv >> 1;
  const int fr = lane & 15, fk = lane >> 4;
  const int sr = tid / TPR, sc = (tid % TPR) * PT;
  const int64_t nslab = a.K / BK;   // even
  const double* yp = a.Y + sr * a.ldy + J0 + sc;
  const double* xq = a.X + (int64_t)fk * a.ldx + I0 + wi * 64 + fr;
  const double* wq = a.w + fk;
  double fy[2][PT];
  auto fload = [&](int64_t s, int h) {
    const double2* ys = reinterpret_cast<const double2*>(yp + s * BK * a.ldy);
#pragma unroll
    for (int q = 0; q < PT / 2; ++q) {
      const double2 v = ys[q];
      fy[h][2 * q] = v.x;
      fy[h][2 * q + 1] = v.y;
    }
  };
  auto fstore = [&](int buf, int h) {
#pragma unroll
    for (int q = 0; q < PT; ++q) sY[buf][sr * LD + sc + q] = fy[h][q];
  };
  double xr[4][TW], wk[4];
  auto xload = [&](int64_t s, int kk) {
    const double* p = xq + (s * BK + kk * 4) * a.ldx;
#pragma unroll
    for (int t = 0; t < TW; ++t) xr[kk][t] = p[t * 16];
    if (WEIGHT) wk[kk] = wq[s * BK + kk * 4];
  };
  dbl4 acc[TW][TW];
#pragma unroll
  for (int u = 0; u < TW; ++u)
#pragma unroll
    for (int v = 0; v < TW; ++v) acc[u][v] = dbl4{0.0, 0.0, 0.0, 0.0};
  fload(0, 0);
  fload(1, 1);
  fstore(0, 0);
  fstore(1, 1);
  fload(std::min<int64_t>(2, nslab - 1), 0);
  fload(std::min<int64_t>(3, nslab - 1), 1);
#pragma unroll
  for (int kk = 0; kk < 4; ++kk) xload(0, kk);
  __syncthreads();
  for (int64_t s = 0; s < nslab; s += 2) {
    const int pb = (int)((s >> 1) & 1) * 2;   // buffers of this pair
    fstore(pb ^ 2, 0);
    fstore((pb ^ 2) + 1, 1);
    fload(std::min<int64_t>(s + 4, nslab - 1), 0);
    fload(std::min<int64_t>(s + 5, nslab - 1), 1);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const double* by = sY[pb + h];
      const int64_t sn = std::min<int64_t>(s + h + 1, nslab - 1);
#pragma unroll
      for (int kk = 0; kk < 4; ++kk) {
        double av[TW], bv[TW];
#pragma unroll
        for (int t = 0; t < TW; ++t) av[t] = by[(kk * 4 + fk) * LD + wj * 64 + t * 16 + fr];
#pragma unroll
        for (int t = 0; t < TW; ++t) bv[t] = WEIGHT ? xr[kk][t] * wk[kk] : xr[kk][t];
        xload(sn, kk);
#pragma unroll
        for (int tj = 0; tj < TW; ++tj)
#pragma unroll
          for (int ti = 0; ti < TW; ++ti)
            acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(av[tj], bv[ti], acc[tj][ti], 0, 0, 0);
      }
    }
    __syncthreads();
  }
  store_tile(a, I0, J0, wi, wj, fr, fk, acc);
}

// the Cholesky's trailing tiles: C -= X^T Y on a lower-triangle grid (LOOP 1 with / without the lazy
// C read, LOOP 2)
template <int LOOP, int LAZYC>
__global__ __launch_bounds__(256, 2) void k_sub(ipm::GemmArgs a) {
  __shared__ ipm::MfSmem<128, 2> sm;
  ipm::mfma_tile<128, false, true, 2, false, false, LOOP, LAZYC>(a, blockIdx.x, sm);
}

static int sub_mode(int64_t n, int64_t K);

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atol(argv[1]) : 8192, K = argc > 2 ? atol(argv[2]) : 2048;
  if (argc > 3) return sub_mode(n, K);
  const int reps = 10;
  double *X, *w, *C, *C0;
  CK(hipMalloc(&X, (size_t)K * n * 8));
  CK(hipMalloc(&w, (size_t)K * 8));
  CK(hipMalloc(&C, (size_t)n * n * 8));
  CK(hipMalloc(&C0, (size_t)n * n * 8));
  {
    std::vector<double> h((size_t)K * n);
    srand(7);
    for (auto& v : h) v = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(X, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> hw(K);
    for (auto& v : hw) v = 0.5 + rand() / (double)RAND_MAX;
    CK(hipMemcpy(w, hw.data(), K * 8, hipMemcpyHostToDevice));
  }
  ipm::GemmArgs a;
  a.ni = a.nj = n; a.K = K; a.X = a.Y = X; a.ldx = a.ldy = n; a.w = w; a.C = C0; a.ldc = n;
  a.alpha = 1.0; a.beta = 0.0; a.tri = 0;
  a.tiles_i = n / BM; a.nblk = a.tiles_i * a.tiles_i;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name, double* out) {
    a.C = out;
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3((unsigned)a.nblk), dim3(256), 0, 0, a);
      hipEventRecord(e1);
      CK(hipEventSynchronize(e1));
      float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    double d = 0.0;
    if (out != C0) {
      std::vector<double> o((size_t)n * n), r((size_t)n * n);
      CK(hipMemcpy(o.data(), out, o.size() * 8, hipMemcpyDeviceToHost));
      CK(hipMemcpy(r.data(), C0, r.size() * 8, hipMemcpyDeviceToHost));
      for (size_t i = 0; i < o.size(); i += 3) d = std::max(d, std::abs(o[i] - r[i]));
    }
    printf("n=%ld K=%ld %-44s median %.3f ms best %.3f  %.1f TF/s  max|dC| vs V0 %.1e\n", (long)n, (long)K, name,
           t[t.size() / 2], t[0], 2.0 * n * n * K / t[t.size() / 2] / 1e9, d);
    fflush(stdout);
  };
  run(k_v0, "V0 library fast loop (weighted)", C0);
  run(k_v1<true>, "V1 X direct to registers (weighted)", C);
  run(k_v6<true>, "V6 V1 + Y fragments one k-step ahead", C);
  run(k_v7<true>, "V7 V1 with two slabs per barrier", C);
  run(k_v1<true>, "V1 again", C);
  run(k_v6<true>, "V6 again", C);
  run(k_v7<true>, "V7 again", C);
  return 0;
}

static int sub_mode(int64_t n, int64_t K) {
  double *X, *C, *C0, *Cs;
  CK(hipMalloc(&X, (size_t)K * n * 8));
  CK(hipMalloc(&C, (size_t)n * n * 8));
  CK(hipMalloc(&C0, (size_t)n * n * 8));
  CK(hipMalloc(&Cs, (size_t)n * n * 8));
  {
    std::vector<double> h((size_t)std::max(K, n) * n);
    srand(9);
    for (size_t i = 0; i < (size_t)K * n; ++i) h[i] = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(X, h.data(), (size_t)K * n * 8, hipMemcpyHostToDevice));
    for (size_t i = 0; i < (size_t)n * n; ++i) h[i] = rand() / (double)RAND_MAX;
    CK(hipMemcpy(Cs, h.data(), (size_t)n * n * 8, hipMemcpyHostToDevice));
  }
  ipm::GemmArgs a;
  a.ni = a.nj = n; a.K = K; a.X = a.Y = X; a.ldx = a.ldy = n; a.ldc = n; a.sub = 1; a.tri = 1;
  a.xcd_remap = 1; a.tiles_i = n / 128; a.nblk = a.tiles_i * (a.tiles_i + 1) / 2;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  std::vector<double> ref;
  auto run = [&](auto kern, const char* name) {
    a.C = C;
    std::vector<float> t;
    for (int r = 0; r < 10; ++r) {
      CK(hipMemcpy(C, Cs, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
      CK(hipDeviceSynchronize());
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3((unsigned)a.nblk), dim3(256), 0, 0, a);
      hipEventRecord(e1);
      CK(hipEventSynchronize(e1));
      float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    std::vector<double> o((size_t)n * n);
    CK(hipMemcpy(o.data(), C, o.size() * 8, hipMemcpyDeviceToHost));
    double d = 0.0;
    if (ref.empty()) ref = o;
    else for (int64_t j = 0; j < n; j += 5) for (int64_t i = j; i < n; ++i) d = std::max(d, std::abs(o[j * n + i] - ref[j * n + i]));
    printf("sub n=%ld K=%ld %-36s median %.1f us best %.1f  %.1f TF/s  max|dC| vs first %.1e\n", (long)n, (long)K, name,
           t[t.size() / 2] * 1e3, t[0] * 1e3, (double)n * (n + 1) * K / t[t.size() / 2] / 1e9, d);
    fflush(stdout);
  };
  run(k_sub<1, 0>, "LOOP 1, C read first");
  run(k_sub<1, 1>, "LOOP 1, lazy C (shipped S tiles)");
  run(k_sub<2, 0>, "LOOP 2, C read first");
  run(k_sub<1, 1>, "LOOP 1 lazy again");
  run(k_sub<2, 0>, "LOOP 2 again");
  return 0;
}
