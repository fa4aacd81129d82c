// fp64 MFMA GEMM lab (not part of the library): C(i,j) = sum_k X[k][i] Y[k][j] on k-major
// operands, lower-triangle (SYRK) or full grids, variants of tile shape / waves / pipeline.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_lab.hip -o tools/gemm_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../interiorpoint-gpu_amd/csrc/ipm_mfma.h"

typedef double dbl4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// BM x BN workgroup tile, WM x WN waves, BK-deep slabs, NSTAGE LDS stages
template <int BM, int BN, int WM, int WN, int BK, bool TRI, int PAD = 0>
__global__ __launch_bounds__(WM * WN * 64) void k_gemm(int n, int K, const double* __restrict__ X, int ldx,
                                                        const double* __restrict__ Y, int ldy,
                                                        double* __restrict__ C, int ldc, int tiles_i, int nblk) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;   // MFMA tiles per wave
  constexpr int LX = BM + 16, LY = BN + 16;              // padded LDS rows
  constexpr int PX = BK * BM / NT, PY = BK * BN / NT;    // doubles per thread per slab
  static_assert(PX % 2 == 0 && PY % 2 == 0, "pairs");
  __shared__ double sX[2][BK * LX];
  __shared__ double sY[2][BK * LY];
  __shared__ double spad[PAD > 0 ? PAD : 1];
  if (PAD > 0 && threadIdx.x == 0 && n < 0) spad[0] = 0.0;   // keep the pad allocated
  for (int Lp = blockIdx.x; Lp < nblk; Lp += gridDim.x) {
  int bi, bj;
  if (TRI) {
    const int L = Lp;
    int b = (int)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while ((b + 1) * (b + 2) / 2 <= L) ++b;
    while (b * (b + 1) / 2 > L) --b;
    bi = b; bj = L - b * (b + 1) / 2;   // BM == BN for TRI
  } else {
    bi = Lp % tiles_i; bj = Lp / tiles_i;
  }
  const int I0 = bi * BM, J0 = bj * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wi = wv % WM, wj = wv / WM;
  dbl4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = dbl4{0, 0, 0, 0};
  // slab staging: thread covers PX consecutive doubles of one X row (and PY of one Y row)
  constexpr int TPRX = BM / PX, TPRY = BN / PY;
  const int xr = tid / TPRX, xc = (tid % TPRX) * PX;
  const int yr = tid / TPRY, yc = (tid % TPRY) * PY;
  double rx[PX], ry[PY];
  auto gload = [&](int k0) {
    const double2* xp = reinterpret_cast<const double2*>(X + (size_t)(k0 + xr) * ldx + I0 + xc);
    const double2* yp = reinterpret_cast<const double2*>(Y + (size_t)(k0 + yr) * ldy + J0 + yc);
#pragma unroll
    for (int q = 0; q < PX / 2; ++q) { double2 v = xp[q]; rx[2 * q] = v.x; rx[2 * q + 1] = v.y; }
#pragma unroll
    for (int q = 0; q < PY / 2; ++q) { double2 v = yp[q]; ry[2 * q] = v.x; ry[2 * q + 1] = v.y; }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < PX; ++q) sX[buf][xr * LX + xc + q] = rx[q];
#pragma unroll
    for (int q = 0; q < PY; ++q) sY[buf][yr * LY + yc + q] = ry[q];
  };
  const int nslab = K / BK;
  gload(0); sstore(0);
  if (nslab > 1) gload(BK);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int s = 0; s < nslab; ++s) {
    const int buf = s & 1;
    const double* bx = sX[buf];
    const double* by = sY[buf];
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[TN], b[TM];
#pragma unroll
      for (int t = 0; t < TN; ++t) a[t] = by[(kk * 4 + fk) * LY + wj * (BN / WN) + t * 16 + fr];
#pragma unroll
      for (int t = 0; t < TM; ++t) b[t] = bx[(kk * 4 + fk) * LX + wi * (BM / WM) + t * 16 + fr];
#pragma unroll
      for (int tj = 0; tj < TN; ++tj)
#pragma unroll
        for (int ti = 0; ti < TM; ++ti) acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[tj], b[ti], acc[tj][ti], 0, 0, 0);
    }
    if (s + 1 < nslab) {
      sstore(buf ^ 1);
      if (s + 2 < nslab) gload((s + 2) * BK);
    }
    __syncthreads();
  }
#pragma unroll
  for (int tj = 0; tj < TN; ++tj)
#pragma unroll
    for (int ti = 0; ti < TM; ++ti) {
      const int i = I0 + wi * (BM / WM) + ti * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = J0 + wj * (BN / WN) + tj * 16 + fk + 4 * r;
        if (!TRI || i >= j) C[(size_t)j * ldc + i] = acc[tj][ti][r];
      }
    }
  __syncthreads();
  }
}

// k_gemm with a branch-free slab loop (one basic block: the slab s+2 loads are issued with the
// slab index clamped, the LDS store of slab s+1 always happens) so that the scheduler can spread
// the LDS reads, the LDS stores and the global loads between the MFMAs; SGB = 1 also pins an
// interleave pattern with sched_group_barrier (mask 0x008 MFMA, 0x100 DS read, 0x200 DS write,
// 0x020 VMEM read, 0x002 VALU)
template <int BM, int BN, int WM, int WN, int BK, int TRI, int SGB>
__global__ __launch_bounds__(WM * WN * 64) void k_gemm2(int n, int K, const double* __restrict__ X, int ldx,
                                                        const double* __restrict__ Y, int ldy,
                                                        double* __restrict__ C, int ldc, int tiles_i, int nblk) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int LX = BM + 16, LY = BN + 16;
  constexpr int PX = BK * BM / NT, PY = BK * BN / NT;
  __shared__ double sX[2][BK * LX];
  __shared__ double sY[2][BK * LY];
  for (int Lp = blockIdx.x; Lp < nblk; Lp += gridDim.x) {
  int bi, bj;
  if (TRI == 1) {          // lower triangle, row-major tile order
    const int L = Lp;
    int b = (int)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while ((b + 1) * (b + 2) / 2 <= L) ++b;
    while (b * (b + 1) / 2 > L) --b;
    bi = b; bj = L - b * (b + 1) / 2;
  } else if (TRI == 2) {   // lower triangle, column-major tile order (bi fastest, as the full grid)
    int L = Lp, c = 0;
    while (L >= tiles_i - c) { L -= tiles_i - c; ++c; }
    bj = c; bi = c + L;
  } else if (TRI == 3) {   // lower triangle, column-major, each XCD a contiguous run
    const int q = nblk >> 3;
    int L = Lp < (q << 3) ? (Lp & 7) * q + (Lp >> 3) : Lp, c = 0;
    while (L >= tiles_i - c) { L -= tiles_i - c; ++c; }
    bj = c; bi = c + L;
  } else {
    bi = Lp % tiles_i; bj = Lp / tiles_i;
  }
  const int I0 = bi * BM, J0 = bj * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wi = wv % WM, wj = wv / WM;
  dbl4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = dbl4{0, 0, 0, 0};
  constexpr int TPRX = BM / PX, TPRY = BN / PY;
  const int xr = tid / TPRX, xc = (tid % TPRX) * PX;
  const int yr = tid / TPRY, yc = (tid % TPRY) * PY;
  double rx[PX], ry[PY];
  const double* xb = X + (size_t)xr * ldx + I0 + xc;
  const double* yb = Y + (size_t)yr * ldy + J0 + yc;
  auto gload = [&](int s) {
    const double2* xp = reinterpret_cast<const double2*>(xb + (size_t)s * BK * ldx);
    const double2* yp = reinterpret_cast<const double2*>(yb + (size_t)s * BK * ldy);
#pragma unroll
    for (int q = 0; q < PX / 2; ++q) { double2 v = xp[q]; rx[2 * q] = v.x; rx[2 * q + 1] = v.y; }
#pragma unroll
    for (int q = 0; q < PY / 2; ++q) { double2 v = yp[q]; ry[2 * q] = v.x; ry[2 * q + 1] = v.y; }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < PX; ++q) sX[buf][xr * LX + xc + q] = rx[q];
#pragma unroll
    for (int q = 0; q < PY; ++q) sY[buf][yr * LY + yc + q] = ry[q];
  };
  const int nslab = K / BK;
  gload(0); sstore(0);
  gload(nslab > 1 ? 1 : 0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int s = 0; s < nslab; ++s) {
    const int buf = s & 1;
    const double* bx = sX[buf];
    const double* by = sY[buf];
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[TN], b[TM];
#pragma unroll
      for (int t = 0; t < TN; ++t) a[t] = by[(kk * 4 + fk) * LY + wj * (BN / WN) + t * 16 + fr];
#pragma unroll
      for (int t = 0; t < TM; ++t) b[t] = bx[(kk * 4 + fk) * LX + wi * (BM / WM) + t * 16 + fr];
#pragma unroll
      for (int tj = 0; tj < TN; ++tj)
#pragma unroll
        for (int ti = 0; ti < TM; ++ti) acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[tj], b[ti], acc[tj][ti], 0, 0, 0);
    }
    sstore(buf ^ 1);                          // slab s+1 (unused after the last slab)
    gload(min(s + 2, nslab - 1));             // slab s+2 (clamped: a harmless reload at the end)
    if (SGB == 1) {
      // per k-step: its LDS reads first, then MFMAs with the stores / loads of the next slabs spread
      constexpr int NM = TN * TM * (BK / 4), NR = (TN + TM) / 2 * (BK / 4);
      constexpr int NW = (PX + PY) / 2, NG = (PX + PY) / 2;
#pragma unroll
      for (int i = 0; i < NM; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
        if (i < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        else if (i - NR < NW) __builtin_amdgcn_sched_group_barrier(0x200, 1, 0);
        else if (i - NR - NW < NG) __builtin_amdgcn_sched_group_barrier(0x020, 1, 0);
      }
    }
    __syncthreads();
  }
#pragma unroll
  for (int tj = 0; tj < TN; ++tj)
#pragma unroll
    for (int ti = 0; ti < TM; ++ti) {
      const int i = I0 + wi * (BM / WM) + ti * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = J0 + wj * (BN / WN) + tj * 16 + fk + 4 * r;
        if (!TRI || i >= j) C[(size_t)j * ldc + i] = acc[tj][ti][r];
      }
    }
  __syncthreads();
  }
}

template <int BM, int BN, int WM, int WN, int BK, bool TRI, int SGB>
__global__ __launch_bounds__(WM * WN * 64, 2) void k_gemm4(int n, int K, const double* __restrict__ X, int ldx,
                                                        const double* __restrict__ Y, int ldy,
                                                        double* __restrict__ C, int ldc, int tiles_i, int nblk) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int LX = BM + 16, LY = BN + 16;
  constexpr int PX = BK * BM / NT, PY = BK * BN / NT;
  __shared__ double sX[2][BK * LX];
  __shared__ double sY[2][BK * LY];
  for (int Lp = blockIdx.x; Lp < nblk; Lp += gridDim.x) {
  int bi, bj;
  if (TRI == 1) {          // lower triangle, row-major tile order
    const int L = Lp;
    int b = (int)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while ((b + 1) * (b + 2) / 2 <= L) ++b;
    while (b * (b + 1) / 2 > L) --b;
    bi = b; bj = L - b * (b + 1) / 2;
  } else if (TRI == 2) {   // lower triangle, column-major tile order (bi fastest, as the full grid)
    int L = Lp, c = 0;
    while (L >= tiles_i - c) { L -= tiles_i - c; ++c; }
    bj = c; bi = c + L;
  } else if (TRI == 3) {   // lower triangle, column-major, each XCD a contiguous run
    const int q = nblk >> 3;
    int L = Lp < (q << 3) ? (Lp & 7) * q + (Lp >> 3) : Lp, c = 0;
    while (L >= tiles_i - c) { L -= tiles_i - c; ++c; }
    bj = c; bi = c + L;
  } else {
    bi = Lp % tiles_i; bj = Lp / tiles_i;
  }
  const int I0 = bi * BM, J0 = bj * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wi = wv % WM, wj = wv / WM;
  dbl4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = dbl4{0, 0, 0, 0};
  constexpr int TPRX = BM / PX, TPRY = BN / PY;
  const int xr = tid / TPRX, xc = (tid % TPRX) * PX;
  const int yr = tid / TPRY, yc = (tid % TPRY) * PY;
  double rx[PX], ry[PY];
  const double* xb = X + (size_t)xr * ldx + I0 + xc;
  const double* yb = Y + (size_t)yr * ldy + J0 + yc;
  auto gload = [&](int s) {
    const double2* xp = reinterpret_cast<const double2*>(xb + (size_t)s * BK * ldx);
    const double2* yp = reinterpret_cast<const double2*>(yb + (size_t)s * BK * ldy);
#pragma unroll
    for (int q = 0; q < PX / 2; ++q) { double2 v = xp[q]; rx[2 * q] = v.x; rx[2 * q + 1] = v.y; }
#pragma unroll
    for (int q = 0; q < PY / 2; ++q) { double2 v = yp[q]; ry[2 * q] = v.x; ry[2 * q + 1] = v.y; }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < PX; ++q) sX[buf][xr * LX + xc + q] = rx[q];
#pragma unroll
    for (int q = 0; q < PY; ++q) sY[buf][yr * LY + yc + q] = ry[q];
  };
  const int nslab = K / BK;
  gload(0); sstore(0);
  gload(nslab > 1 ? 1 : 0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int s = 0; s < nslab; ++s) {
    const int buf = s & 1;
    const double* bx = sX[buf];
    const double* by = sY[buf];
    // SGB 2: the whole slab's operand fragments first (all 4 k-steps), then the stores / loads of
    // the next slabs, then the 64 MFMAs from registers
    double a[BK / 4][TN], b[BK / 4][TM];
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
#pragma unroll
      for (int t = 0; t < TN; ++t) a[kk][t] = by[(kk * 4 + fk) * LY + wj * (BN / WN) + t * 16 + fr];
#pragma unroll
      for (int t = 0; t < TM; ++t) b[kk][t] = bx[(kk * 4 + fk) * LX + wi * (BM / WM) + t * 16 + fr];
    }
    sstore(buf ^ 1);
    gload(min(s + 2, nslab - 1));
    if (SGB == 2) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk)
#pragma unroll
      for (int tj = 0; tj < TN; ++tj)
#pragma unroll
        for (int ti = 0; ti < TM; ++ti) acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[kk][tj], b[kk][ti], acc[tj][ti], 0, 0, 0);
    __syncthreads();
  }
#pragma unroll
  for (int tj = 0; tj < TN; ++tj)
#pragma unroll
    for (int ti = 0; ti < TM; ++ti) {
      const int i = I0 + wi * (BM / WM) + ti * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = J0 + wj * (BN / WN) + tj * 16 + fk + 4 * r;
        if (!TRI || i >= j) C[(size_t)j * ldc + i] = acc[tj][ti][r];
      }
    }
  __syncthreads();
  }
}

// k_gemm2 with the slabs brought into LDS by the load itself (global_load_lds, 16 bytes per lane:
// one wave instruction = one 128-double slab row): no register staging, no LDS store
// instructions.  One slab of prefetch (the DMA of slab s+1 runs under slab s's MFMAs).
template <int BM, int BN, int BK, bool TRI>
__global__ __launch_bounds__(256, 2) void k_gemm3(int n, int K, const double* __restrict__ X, int ldx,
                                                 const double* __restrict__ Y, int ldy,
                                                 double* __restrict__ C, int ldc, int tiles_i, int nblk) {
  constexpr int WM = 2, WN = 2;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;
  constexpr int LX = BM + 16, LY = BN + 16;
  static_assert(BM == 128 && BN == 128, "one wave instruction per slab row");
  __shared__ double sX[2][BK * LX];
  __shared__ double sY[2][BK * LY];
  for (int Lp = blockIdx.x; Lp < nblk; Lp += gridDim.x) {
  int bi, bj;
  if (TRI) {
    const int L = Lp;
    int b = (int)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while ((b + 1) * (b + 2) / 2 <= L) ++b;
    while (b * (b + 1) / 2 > L) --b;
    bi = b; bj = L - b * (b + 1) / 2;
  } else {
    bi = Lp % tiles_i; bj = Lp / tiles_i;
  }
  const int I0 = bi * BM, J0 = bj * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wi = wv % WM, wj = wv / WM;
  dbl4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = dbl4{0, 0, 0, 0};
  // wave wv loads slab rows wv, wv+4, wv+8, wv+12 of both operands: 8 instructions per slab
  auto dma = [&](int s, int buf) {
#pragma unroll
    for (int r = 0; r < BK / 4; ++r) {
      const int row = wv + 4 * r;
      const double* gx = X + (size_t)(s * BK + row) * ldx + I0 + 2 * lane;
      const double* gy = Y + (size_t)(s * BK + row) * ldy + J0 + 2 * lane;
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gx,
                                       (__attribute__((address_space(3))) void*)&sX[buf][row * LX], 16, 0, 0);
      __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)gy,
                                       (__attribute__((address_space(3))) void*)&sY[buf][row * LY], 16, 0, 0);
    }
  };
  const int nslab = K / BK;
  dma(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int s = 0; s < nslab; ++s) {
    const int buf = s & 1;
    dma(min(s + 1, nslab - 1), buf ^ 1);      // slab s+1 (a harmless reload after the last)
    const double* bx = sX[buf];
    const double* by = sY[buf];
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[TN], b[TM];
#pragma unroll
      for (int t = 0; t < TN; ++t) a[t] = by[(kk * 4 + fk) * LY + wj * (BN / WN) + t * 16 + fr];
#pragma unroll
      for (int t = 0; t < TM; ++t) b[t] = bx[(kk * 4 + fk) * LX + wi * (BM / WM) + t * 16 + fr];
#pragma unroll
      for (int tj = 0; tj < TN; ++tj)
#pragma unroll
        for (int ti = 0; ti < TM; ++ti) acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[tj], b[ti], acc[tj][ti], 0, 0, 0);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
#pragma unroll
  for (int tj = 0; tj < TN; ++tj)
#pragma unroll
    for (int ti = 0; ti < TM; ++ti) {
      const int i = I0 + wi * (BM / WM) + ti * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = J0 + wj * (BN / WN) + tj * 16 + fk + 4 * r;
        if (!TRI || i >= j) C[(size_t)j * ldc + i] = acc[tj][ti][r];
      }
    }
  __syncthreads();
  }
}

__global__ void k_ref(int n, int K, const double* X, int ldx, const double* Y, int ldy, double* C, int ldc) {
  int i = blockIdx.x * 256 + threadIdx.x, j = blockIdx.y;
  if (i >= n) return;
  double s = 0;
  for (int k = 0; k < K; ++k) s = fma(X[(size_t)k * ldx + i], Y[(size_t)k * ldy + j], s);
  C[(size_t)j * ldc + i] = s;
}

template <int BM, int BN, int WM, int WN, int BK, bool TRI, int PAD = 0>
void run(const char* name, int n, int K, double* X, double* Y, double* C, double* R, int reps, int grid = 0) {
  const int ti = n / BM, tj = n / BN;
  const int nblk = TRI ? ti * (ti + 1) / 2 : ti * tj;
  auto launch = [&]() {
    hipLaunchKernelGGL((k_gemm<BM, BN, WM, WN, BK, TRI, PAD>), dim3(grid ? grid : nblk), dim3(WM * WN * 64), 0, 0, n, K, X, n, Y, n, C, n, ti, nblk);
  };
  CK(hipMemset(C, 0, (size_t)n * n * 8));
  launch();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float best = 1e30, tot = 0;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); best = std::min(best, ms); tot += ms;
  }
  // check a sample of columns
  std::vector<double> hc((size_t)n * n), hr((size_t)n * n);
  CK(hipMemcpy(hc.data(), C, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), R, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  double err = 0, mx = 0;
  for (int j = 0; j < n; j += 97)
    for (int i = TRI ? j : 0; i < n; ++i) { err = std::max(err, fabs(hc[(size_t)j * n + i] - hr[(size_t)j * n + i])); mx = std::max(mx, fabs(hr[(size_t)j * n + i])); }
  const double fl = TRI ? (double)n * (n + 1) * K : 2.0 * n * n * K;  // tri: useful flops of the triangle
  printf("%-34s n=%d K=%d blocks=%6d  best %.3f ms avg %.3f  %.1f TF/s  relerr %.1e\n", name, n, K, nblk, best,
         tot / reps, fl / best / 1e9, err / mx);
}

template <int BM, int BN, int WM, int WN, int BK, int TRI, int SGB>
void run2(const char* name, int n, int K, double* X, double* Y, double* C, double* R, int reps, int grid = 0) {
  const int ti = n / BM, tj = n / BN;
  const int nblk = TRI ? ti * (ti + 1) / 2 : ti * tj;
  auto launch = [&]() {
    hipLaunchKernelGGL((k_gemm2<BM, BN, WM, WN, BK, TRI, SGB>), dim3(grid ? grid : nblk), dim3(WM * WN * 64), 0, 0, n, K, X, n, Y, n, C, n, ti, nblk);
  };
  CK(hipMemset(C, 0, (size_t)n * n * 8));
  launch();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float best = 1e30, tot = 0;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); best = std::min(best, ms); tot += ms;
  }
  // check a sample of columns
  std::vector<double> hc((size_t)n * n), hr((size_t)n * n);
  CK(hipMemcpy(hc.data(), C, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), R, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  double err = 0, mx = 0;
  for (int j = 0; j < n; j += 97)
    for (int i = TRI ? j : 0; i < n; ++i) { err = std::max(err, fabs(hc[(size_t)j * n + i] - hr[(size_t)j * n + i])); mx = std::max(mx, fabs(hr[(size_t)j * n + i])); }
  const double fl = TRI ? (double)n * (n + 1) * K : 2.0 * n * n * K;  // tri: useful flops of the triangle
  printf("%-34s n=%d K=%d blocks=%6d  best %.3f ms avg %.3f  %.1f TF/s  relerr %.1e\n", name, n, K, nblk, best,
         tot / reps, fl / best / 1e9, err / mx);
}

template <int BM, int BN, int WM, int WN, int BK, bool TRI>
void run3(const char* name, int n, int K, double* X, double* Y, double* C, double* R, int reps, int grid = 0) {
  const int ti = n / BM, tj = n / BN;
  const int nblk = TRI ? ti * (ti + 1) / 2 : ti * tj;
  auto launch = [&]() {
    hipLaunchKernelGGL((k_gemm3<BM, BN, BK, TRI>), dim3(grid ? grid : nblk), dim3(WM * WN * 64), 0, 0, n, K, X, n, Y, n, C, n, ti, nblk);
  };
  CK(hipMemset(C, 0, (size_t)n * n * 8));
  launch();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float best = 1e30, tot = 0;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); best = std::min(best, ms); tot += ms;
  }
  // check a sample of columns
  std::vector<double> hc((size_t)n * n), hr((size_t)n * n);
  CK(hipMemcpy(hc.data(), C, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), R, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  double err = 0, mx = 0;
  for (int j = 0; j < n; j += 97)
    for (int i = TRI ? j : 0; i < n; ++i) { err = std::max(err, fabs(hc[(size_t)j * n + i] - hr[(size_t)j * n + i])); mx = std::max(mx, fabs(hr[(size_t)j * n + i])); }
  const double fl = TRI ? (double)n * (n + 1) * K : 2.0 * n * n * K;  // tri: useful flops of the triangle
  printf("%-34s n=%d K=%d blocks=%6d  best %.3f ms avg %.3f  %.1f TF/s  relerr %.1e\n", name, n, K, nblk, best,
         tot / reps, fl / best / 1e9, err / mx);
}

template <int BM, int BN, int WM, int WN, int BK, bool TRI, int SGB>
void run4(const char* name, int n, int K, double* X, double* Y, double* C, double* R, int reps, int grid = 0) {
  const int ti = n / BM, tj = n / BN;
  const int nblk = TRI ? ti * (ti + 1) / 2 : ti * tj;
  auto launch = [&]() {
    hipLaunchKernelGGL((k_gemm4<BM, BN, WM, WN, BK, TRI, SGB>), dim3(grid ? grid : nblk), dim3(WM * WN * 64), 0, 0, n, K, X, n, Y, n, C, n, ti, nblk);
  };
  CK(hipMemset(C, 0, (size_t)n * n * 8));
  launch();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float best = 1e30, tot = 0;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); best = std::min(best, ms); tot += ms;
  }
  // check a sample of columns
  std::vector<double> hc((size_t)n * n), hr((size_t)n * n);
  CK(hipMemcpy(hc.data(), C, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), R, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  double err = 0, mx = 0;
  for (int j = 0; j < n; j += 97)
    for (int i = TRI ? j : 0; i < n; ++i) { err = std::max(err, fabs(hc[(size_t)j * n + i] - hr[(size_t)j * n + i])); mx = std::max(mx, fabs(hr[(size_t)j * n + i])); }
  const double fl = TRI ? (double)n * (n + 1) * K : 2.0 * n * n * K;  // tri: useful flops of the triangle
  printf("%-34s n=%d K=%d blocks=%6d  best %.3f ms avg %.3f  %.1f TF/s  relerr %.1e\n", name, n, K, nblk, best,
         tot / reps, fl / best / 1e9, err / mx);
}

void runlib(const char* name, int n, int K, bool tri, bool weight, int remap, double* X, double* C, double* R,
            double* w, int reps, int persist = 0, double beta = 0.0) {
  ipm::GemmArgs a;
  a.ni = n; a.nj = n; a.K = K; a.X = X; a.ldx = n; a.Y = X; a.ldy = n; a.w = weight ? w : nullptr;
  a.C = C; a.ldc = n; a.tri = tri; a.xcd_remap = remap; a.beta = beta; if (beta == 1.0) a.alpha = -1.0;
  CK(hipMemset(C, 0, (size_t)n * n * 8));
  auto L = [&]() { if (persist) ipm::mfma_gemm_launch_persistent(0, a, persist); else ipm::mfma_gemm_launch(0, a); };
  L();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float best = 1e30, tot = 0;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0)); L(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms); tot += ms;
  }
  std::vector<double> hc((size_t)n * n), hr((size_t)n * n);
  CK(hipMemcpy(hc.data(), C, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), R, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  double err = 0, mx = 0;
  if (!weight && beta == 0.0)
    for (int j = 0; j < n; j += 97)
      for (int i = tri ? j : 0; i < n; ++i) { err = std::max(err, fabs(hc[(size_t)j * n + i] - hr[(size_t)j * n + i])); mx = std::max(mx, fabs(hr[(size_t)j * n + i])); }
  const double fl = tri ? (double)n * (n + 1) * K : 2.0 * n * n * K;
  printf("%-34s n=%d K=%d  best %.3f ms avg %.3f  %.1f TF/s  relerr %.1e\n", name, n, K, best, tot / reps, fl / best / 1e9,
         mx > 0 ? err / mx : 0.0);
}

// the library's KKT SYRK launch (mfma_gemm_launch_split: stream-K tail) with the pieces of the KKT
// assembly switched on one at a time: the weight on k, the tP * P epilogue, the diagonal vector
void runsyrk(const char* name, int n, int K, bool weight, bool pepi, double* X, double* C, double* w, double* P,
             double* dv, int reps) {
  ipm::GemmArgs a;
  a.ni = a.nj = n; a.K = K; a.X = a.Y = X; a.ldx = a.ldy = n; a.w = weight ? w : nullptr;
  a.C = C; a.ldc = n; a.tri = 1; a.alpha = 1.0; a.beta = 0.0;
  if (pepi) { a.P = P; a.ldp = n; a.tP = 0.5; a.dvec = dv; }
  const int64_t cap = ipm::syrk_split_cap(n);
  double* ws; CK(hipMalloc(&ws, ipm::syrk_split_ws_doubles(n) * 8));
  int ncu = 0; CK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0));
  auto L = [&]() { ipm::mfma_gemm_launch_split(0, a, ws, cap, 2 * ncu); };
  L();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float best = 1e30, tot = 0;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0)); L(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms); tot += ms;
  }
  const double fl = (double)n * (n + 1) * K;
  printf("%-34s n=%d K=%d  best %.3f ms avg %.3f  %.1f TF/s\n", name, n, K, best, tot / reps, fl / best / 1e9);
  CK(hipFree(ws));
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 8192;
  const int K = argc > 2 ? atoi(argv[2]) : 2048;
  double *X, *C, *R;
  CK(hipMalloc(&X, (size_t)K * n * 8)); CK(hipMalloc(&C, (size_t)n * n * 8)); CK(hipMalloc(&R, (size_t)n * n * 8));
  std::vector<double> hx((size_t)K * n);
  srand(1);
  for (auto& v : hx) v = (rand() / (double)RAND_MAX) * 4 - 2;
  CK(hipMemcpy(X, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_ref, dim3(n / 256, n), dim3(256), 0, 0, n, K, X, n, X, n, R, n);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  double* w; CK(hipMalloc(&w, (size_t)K * 8));
  { std::vector<double> hw(K, 1.5); CK(hipMemcpy(w, hw.data(), K * 8, hipMemcpyHostToDevice)); }
  if (argc > 3 && atoi(argv[3]) == 1) {   // the library SYRK only (IPM_STREAMK picks its tail)
    double *P, *dv; CK(hipMalloc(&P, (size_t)n * n * 8)); CK(hipMalloc(&dv, (size_t)n * 8));
    CK(hipMemset(P, 0, (size_t)n * n * 8)); CK(hipMemset(dv, 0, (size_t)n * 8));
    for (int rep = 0; rep < 3; ++rep) runsyrk("lib syrk + weight + tP/dvec", n, K, true, true, X, C, w, P, dv, 8);
    return 0;
  }
  runlib("lib tri remap", n, K, true, false, 1, X, C, R, w, reps);
  run2<128, 128, 2, 2, 16, true, 0>("lab2 128x128 w2x2 bk16 tri", n, K, X, X, C, R, reps);
  run4<128, 128, 2, 2, 16, true, 0>("lab4 reads-first tri", n, K, X, X, C, R, reps);
  run4<128, 128, 2, 2, 16, true, 2>("lab4 reads-first+sb tri", n, K, X, X, C, R, reps);
  run2<128, 128, 2, 2, 16, false, 0>("lab2 128x128 w2x2 bk16 full", n, K, X, X, C, R, reps);
  run4<128, 128, 2, 2, 16, false, 0>("lab4 reads-first full", n, K, X, X, C, R, reps);
  run4<128, 128, 2, 2, 16, false, 2>("lab4 reads-first+sb full", n, K, X, X, C, R, reps);
  // round 4 (profiles/r4h_gemm_lab.txt): larger tiles were slower (256x128 w2x2: 53-62 TF/s,
  // 256x128 w4x2 59.9, 128x256 54.2, 256x256 spills); the lower-triangle grid's rounds run ~16 %
  // slower than the full grid's: tile orders of the triangle
  {
    double *P, *dv; CK(hipMalloc(&P, (size_t)n * n * 8)); CK(hipMalloc(&dv, (size_t)n * 8));
    CK(hipMemset(P, 0, (size_t)n * n * 8)); CK(hipMemset(dv, 0, (size_t)n * 8));
    for (int rep = 0; rep < 2; ++rep) {
      runsyrk("lib syrk stream-K", n, K, false, false, X, C, w, P, dv, reps);
      runsyrk("lib syrk stream-K + weight", n, K, true, false, X, C, w, P, dv, reps);
      runsyrk("lib syrk stream-K + weight + tP/dvec", n, K, true, true, X, C, w, P, dv, reps);
    }
    CK(hipFree(P)); CK(hipFree(dv));
  }
  run2<128, 128, 2, 2, 16, 2, 0>("lab2 tri column-major", n, K, X, X, C, R, reps);
  run2<128, 128, 2, 2, 16, 3, 0>("lab2 tri column-major xcd runs", n, K, X, X, C, R, reps);
  run2<128, 128, 2, 2, 16, 1, 0>("lab2 tri row-major (again)", n, K, X, X, C, R, reps);
  return 0;
}
