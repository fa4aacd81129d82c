// Micro-benchmark of the 16x16 Cholesky leaf (diagonal role, wave 0) in isolation: one wave,
// data in registers, N repetitions; cycles per leaf from s_memtime.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#include <algorithm>
#define IPM_STAMPS 1
#include "../interiorpoint-gpu_amd/csrc/ipm_blas.hip"

__device__ __forceinline__ double dpp_bcast(double x, int l) {
  switch (l) {
#define C(k) case k: return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + k, 0xf, 0xf, false);
    C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15)
#undef C
  }
  return 0.0;
}

template <int V>
__global__ __launch_bounds__(64) void k_leaf(double* io, unsigned long long* cyc, int reps) {
  const int lane = threadIdx.x & 63, rr = lane & 15;
  double row[16];
  for (int c = 0; c < 16; ++c) row[c] = io[c * 16 + rr];
  const double keep0 = row[0];
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  double acc = 0.0;
  for (int it = 0; it < reps; ++it) {
    int bad = 0;
    double piv = ipm::readlane_d(row[0], 0);
    double dv = ipm::rsqrt_pivot(piv);
    double dvs[16];
    if (V == 1) {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (!(piv > 0.0) && bad == 0) bad = c + 1;
        dvs[c] = dv;
        row[c] *= dv;
        double l[16];
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) l[c2] = ipm::readlane_d(row[c], c2);
        double pivn = 1.0, dvn = 1.0;
        if (c + 1 < 16) {
          row[c + 1] = fma(-row[c], l[c + 1], row[c + 1]);
          pivn = ipm::readlane_d(row[c + 1], c + 1);
          dvn = ipm::rsqrt_pivot(pivn);
        }
#pragma unroll
        for (int c2 = c + 2; c2 < 16; ++c2) row[c2] = fma(-row[c], l[c2], row[c2]);
        piv = pivn;
        dv = dvn;
      }
    } else if (V == 4 || V == 5) {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (!(piv > 0.0) && bad == 0) bad = c + 1;
        dvs[c] = dv;
        double pivn = 1.0, dvn = 1.0;
        if (c + 1 < 16) {
          const double a1 = ipm::readlane_d(row[c], c + 1);
          const double d1 = ipm::readlane_d(row[c + 1], c + 1);
          const double l1 = a1 * dv;
          pivn = fma(-l1, l1, d1);
          dvn = V == 5 ? __builtin_amdgcn_rsq(pivn) : ipm::rsqrt_pivot(pivn);
        }
        row[c] *= dv;
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) ipm::fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
        piv = pivn;
        dv = dvn;
      }
    } else if (V == 9 || V == 10) {
      // the diag_role leaf as shipped: diagonal tile rows + the tile-below rows (rowb), one sweep;
      // V == 10: no tile-below rows (their updates move elsewhere)
      double rowb[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) rowb[c] = row[c] * 0.5;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (!(piv > 0.0) && bad == 0) bad = c + 1;
        dvs[c] = dv;
        double pivn = 1.0, dvn = 1.0;
        if (c + 1 < 16) {
          const double a1 = ipm::readlane_d(row[c], c + 1);
          const double d1 = ipm::readlane_d(row[c + 1], c + 1);
          const double l1 = a1 * dv;
          pivn = fma(-l1, l1, d1);
          dvn = ipm::rsqrt_pivot(pivn);
        }
        row[c] *= dv;
        if (V == 9) rowb[c] *= dv;
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) {
          ipm::fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
          if (V == 9) ipm::fmac_bcast16(rowb[c2], row[c], rowb[c], c2, false);
        }
        piv = pivn;
        dv = dvn;
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) acc += rowb[c];
    } else if (V == 11 || V == 12) {
      // V == 4 with the DPP broadcasts as compiler builtins (schedulable; the DPP combiner may fold
      // them into v_fmac_f64_dpp); V == 12 also with tile-below rows
      double rowb[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) rowb[c] = row[c] * 0.5;
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        if (!(piv > 0.0) && bad == 0) bad = c + 1;
        dvs[c] = dv;
        double pivn = 1.0, dvn = 1.0;
        if (c + 1 < 16) {
          const double a1 = ipm::readlane_d(row[c], c + 1);
          const double d1 = ipm::readlane_d(row[c + 1], c + 1);
          const double l1 = a1 * dv;
          pivn = fma(-l1, l1, d1);
          dvn = ipm::rsqrt_pivot(pivn);
        }
        row[c] *= dv;
        if (V == 12) rowb[c] *= dv;
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) {
          const double b = dpp_bcast(row[c], c2);
          row[c2] = fma(-b, row[c], row[c2]);
          if (V == 12) rowb[c2] = fma(-b, rowb[c], rowb[c2]);
        }
        piv = pivn;
        dv = dvn;
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) acc += rowb[c];
    } else if (V == 13 || V == 14) {
      // the shipped DPP leaf with the pivot chain of column c+1 interleaved instruction by
      // instruction with column c's rank-1 updates (sched_barrier pins the order); V == 14 also
      // with the tile-below rows
      double rowb[16];
#pragma unroll
      for (int c = 0; c < 16; ++c) rowb[c] = row[c] * 0.5;
#define SB() __builtin_amdgcn_sched_barrier(0)
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        dvs[c] = dv;
        double a1 = 0.0, d1 = 1.0;
        if (c + 1 < 16) {
          a1 = ipm::readlane_d(row[c], c + 1);
          d1 = ipm::readlane_d(row[c + 1], c + 1);
        }
        row[c] *= dv;
        if (V == 14) rowb[c] *= dv;
        SB();
        double l1 = 0.0, pivn = 1.0, y0 = 1.0, tt = 0.0, e = 0.0, hh = 0.0, gg = 0.0, dvn = 1.0;
        int step = 0;
        auto chain = [&](int k) {
          if (c + 1 >= 16) return;
          switch (k) {
            case 0: l1 = a1 * dv; break;
            case 1: pivn = fma(-l1, l1, d1); break;
            case 2: y0 = __builtin_amdgcn_rsq(pivn); break;
            case 3: tt = pivn * y0; break;
            case 4: e = fma(-tt, y0, 1.0); break;
            case 5: hh = fma(e, 0.375, 0.5); gg = y0 * e; break;
            case 6: dvn = fma(gg, hh, y0); break;
          }
        };
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) {
          if (step < 7) { chain(step++); SB(); }
          ipm::fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
          if (V == 14) ipm::fmac_bcast16(rowb[c2], row[c], rowb[c], c2, false);
          SB();
        }
        while (step < 7) { chain(step++); SB(); }
        if (!(piv > 0.0) && bad == 0) bad = c + 1;
        piv = pivn;
        dv = dvn;
      }
#undef SB
#pragma unroll
      for (int c = 0; c < 16; ++c) acc += rowb[c];
    } else if (V == 6) {
      // chain only: pivots, no vector updates
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        dvs[c] = dv;
        const double a1 = ipm::readlane_d(row[c], (c + 1) & 15);
        const double l1 = a1 * dv;
        const double pivn = fma(-l1, l1, piv + 1.0);
        dv = ipm::rsqrt_pivot(pivn);
        piv = pivn;
      }
    } else if (V == 7) {
      // vector updates only (DPP), no chain
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        row[c] *= dv;
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) ipm::fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
      }
    }
    for (int c = 0; c < 16; ++c) acc += dvs[c] + row[c];
    if (reps == 1) break;
    for (int c = 0; c < 16; ++c) row[c] = (c == 0) ? keep0 : row[c] * 1e-300 + io[c * 16 + rr];
    acc += bad;
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[0] = (t1 - t0) / reps;
  io[256 + lane] = acc;
  if (reps == 1 && lane < 16)
    for (int c = 0; c < 16; ++c) io[320 + c * 16 + lane] = row[c];
}

int main() {
  std::vector<double> h(256 + 64 + 256);
  for (int c = 0; c < 16; ++c)
    for (int r = 0; r < 16; ++r) h[c * 16 + r] = (r == c) ? 40.0 : 0.1 / (1 + r + c);
  double* io; unsigned long long* cyc;
  hipMalloc(&io, h.size() * 8); hipMalloc(&cyc, 8);
  auto run = [&](auto kern, const char* name) {
    hipMemcpy(io, h.data(), h.size() * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, io, cyc, 200);
    unsigned long long c; hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-40s %6llu cycles per leaf (incl. reset loop)\n", name, c);
  };
  // correctness: one leaf, V=1 (readlane) vs V=4/5 (DPP) on the same SPD tile
  {
    std::vector<double> r1(256), r4(256);
    auto one = [&](auto kern, std::vector<double>& out) {
      hipMemcpy(io, h.data(), h.size() * 8, hipMemcpyHostToDevice);
      hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, io, cyc, 1);
      std::vector<double> o(h.size());
      hipMemcpy(o.data(), io, o.size() * 8, hipMemcpyDeviceToHost);
      for (int i = 0; i < 256; ++i) out[i] = o[320 + i];
    };
    one(k_leaf<13>, r1);
    one(k_leaf<4>, r4);
    double md = 0;
    for (int c = 0; c < 16; ++c)
      for (int r = c; r < 16; ++r) md = std::max(md, std::abs(r1[c * 16 + r] - r4[c * 16 + r]));
    printf("max |L(interleaved) - L(dpp)| over the lower triangle: %.3e\n", md);
  }
  run(k_leaf<1>, "readlane broadcasts");
  run(k_leaf<4>, "DPP updates + minimal chain");
  run(k_leaf<5>, "DPP + minimal chain, bare rsq");
  run(k_leaf<9>, "shipped leaf (diag + tile-below rows)");
  run(k_leaf<10>, "shipped leaf, diag rows only");
  run(k_leaf<11>, "builtin DPP, diag rows only");
  run(k_leaf<12>, "builtin DPP, diag + tile-below rows");
  run(k_leaf<13>, "interleaved chain, diag rows only");
  run(k_leaf<14>, "interleaved chain, diag + tile-below rows");
  run(k_leaf<6>, "pivot chain only");
  run(k_leaf<7>, "DPP vector updates only");
  return 0;
}
