// Micro-benchmark of the 16x16 Cholesky leaf (diagonal role, wave 0) in isolation: one wave,
// data in registers, N repetitions; cycles per leaf from s_memtime.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include <cmath>
#include <algorithm>
#define IPM_STAMPS 1
#include "../interiorpoint-gpu_amd/csrc/ipm_blas.hip"

template <int V>
__global__ void k_leaf(double* io, unsigned long long* cyc, int reps) {
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
    one(k_leaf<1>, r1);
    one(k_leaf<4>, r4);
    double md = 0;
    for (int c = 0; c < 16; ++c)
      for (int r = c; r < 16; ++r) md = std::max(md, std::abs(r1[c * 16 + r] - r4[c * 16 + r]));
    printf("max |L(readlane) - L(dpp)| over the lower triangle: %.3e\n", md);
  }
  run(k_leaf<1>, "readlane broadcasts");
  run(k_leaf<4>, "DPP updates + minimal chain");
  run(k_leaf<5>, "DPP + minimal chain, bare rsq");
  run(k_leaf<6>, "pivot chain only");
  run(k_leaf<7>, "DPP vector updates only");
  return 0;
}
