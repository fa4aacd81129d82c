// The 16-column Cholesky leaf sweep (ipm::diag_role's step 2) in isolation, in several instruction
// forms (diagnostic only, never part of the library).  One wave, registers only, the sweep repeated
// `reps` times with an exact restore; prints cycles per sweep and the largest difference of the
// solved tile rows against the shipped form F0 (all forms do the same fma operations: expected 0).
//   F0 shipped: two register streams per lane -- the diagonal rows (a copy in each 16-lane group)
//      and one tile-below row -- each updated by v_fmac_f64_dpp row_newbcast (DPP src0 = column c)
//   F1 two streams, the multiplier L[c2][c] broadcast once per (c, c2) as two 32-bit DPP movs,
//      then two plain v_fma_f64
//   F2 two streams, the multiplier through an SGPR pair (2 x v_readlane_b32), two plain v_fma_f64
//   F3 ONE stream: lane group 0 = the diagonal rows, groups 1-3 = tile rows, multiplier through an
//      SGPR pair, one v_fma_f64 per (c, c2)
//   F4 two streams, the multiplier as one v_mov_b64_dpp (builtin update_dpp), two plain v_fma_f64
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off -Iinteriorpoint-gpu_amd/csrc
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include <algorithm>

__device__ __forceinline__ double readlane_d(double v, int l) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), l);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), l);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double rsqrt_pivot(double x) {
  const double y0 = __builtin_amdgcn_rsq(x);
  const double e = fma(-x * y0, y0, 1.0);
  return fma(y0 * e, fma(e, 0.375, 0.5), y0);
}
#define CASES(M) M(0) M(1) M(2) M(3) M(4) M(5) M(6) M(7) M(8) M(9) M(10) M(11) M(12) M(13) M(14) M(15)
__device__ __forceinline__ void fmac_dpp(double& acc, double xb, double x, int l) {
  switch (l) {
#define C(k) case k: asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:" #k " row_mask:0xf bank_mask:0xf" : "+v"(acc) : "v"(xb), "v"(x)); break;
    CASES(C)
#undef C
  }
}
__device__ __forceinline__ double bcast32x2(double x, int l) {
  int lo = __double2loint(x), hi = __double2hiint(x);
  switch (l) {
#define C(k) case k: lo = __builtin_amdgcn_update_dpp(0, lo, 0x150 + k, 0xf, 0xf, false); hi = __builtin_amdgcn_update_dpp(0, hi, 0x150 + k, 0xf, 0xf, false); break;
    CASES(C)
#undef C
  }
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double bcast64(double x, int l) {
  switch (l) {
#define C(k) case k: return __builtin_amdgcn_update_dpp(0.0, x, 0x150 + k, 0xf, 0xf, false);
    CASES(C)
#undef C
  }
  return 0.0;
}

template <int F>
__global__ __launch_bounds__(64) void k_sweep(const double* io, double* out, unsigned long long* cyc, int reps) {
  const int lane = threadIdx.x & 63, rr = lane & 15, g = lane >> 4;
  const double zero = io[1024];   // 0.0 at run time: the restore is exact
  double orig[16], origb[16], row[16], rowb[16];
  for (int c = 0; c < 16; ++c) {
    if (F == 3) {
      orig[c] = io[(g == 0 ? 0 : 256 * g) + c * 16 + rr];   // group 0 diagonal rows, 1-3 tiles 1-3
      origb[c] = 0.0;
    } else {
      orig[c] = io[c * 16 + rr];                    // diagonal rows (a copy per group)
      origb[c] = io[256 * (g + 1) + c * 16 + rr];   // group g: tile g + 1 (tile 4 is tile 1's copy)
    }
    row[c] = orig[c];
    rowb[c] = origb[c];
  }
  double acc = 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < reps; ++it) {
    double piv = readlane_d(row[0], 0);
    double dv = rsqrt_pivot(piv);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      acc += dv;
      double pivn = 1.0, dvn = 1.0;
      if (c + 1 < 16) {
        const double a1 = readlane_d(row[c], c + 1);
        const double d1 = readlane_d(row[c + 1], c + 1);
        const double l1 = a1 * dv;
        pivn = fma(-l1, l1, d1);
        dvn = rsqrt_pivot(pivn);
      }
      row[c] *= dv;
      if (F != 3) rowb[c] *= dv;
#pragma unroll
      for (int c2 = c + 1; c2 < 16; ++c2) {
        if (F == 0) {
          fmac_dpp(row[c2], row[c], row[c], c2);
          fmac_dpp(rowb[c2], row[c], rowb[c], c2);
        } else if (F == 1) {
          const double m = bcast32x2(row[c], c2);
          row[c2] = fma(-m, row[c], row[c2]);
          rowb[c2] = fma(-m, rowb[c], rowb[c2]);
        } else if (F == 2) {
          const double m = readlane_d(row[c], c2);
          row[c2] = fma(-m, row[c], row[c2]);
          rowb[c2] = fma(-m, rowb[c], rowb[c2]);
        } else if (F == 3) {
          const double m = readlane_d(row[c], c2);
          row[c2] = fma(-m, row[c], row[c2]);
        } else if (F == 4) {
          const double m = bcast64(row[c], c2);
          row[c2] = fma(-m, row[c], row[c2]);
          rowb[c2] = fma(-m, rowb[c], rowb[c2]);
        }
      }
      piv = pivn;
      dv = dvn;
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {   // restore (keeps a dependence on the sweep's result)
      acc += row[c] + rowb[c];
      row[c] = fma(row[c], zero, orig[c]);
      rowb[c] = fma(rowb[c], zero, origb[c]);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[0] = (t1 - t0) / reps;
  out[lane] = acc;
  if (reps == 1) {
    // solved rows of tiles 1..3 -> out[64 + 256 (t - 1) + 16 c + r]
    for (int c = 0; c < 16; ++c) {
      if (F == 3) {
        if (g > 0) out[64 + 256 * (g - 1) + 16 * c + rr] = row[c];
      } else {
        if (g < 3) out[64 + 256 * g + 16 * c + rr] = rowb[c];
      }
    }
  }
}

int main() {
  const int n = 80;   // diagonal block + 4 tiles below (rows 16..79), SPD
  std::vector<double> M((size_t)(n + 8) * n), h((size_t)n * n);
  srand(7);
  for (auto& v : M) v = rand() / (double)RAND_MAX - 0.5;
  for (int j = 0; j < n; ++j)
    for (int i = 0; i < n; ++i) {
      double s = (i == j) ? 4.0 : 0.0;
      for (int k = 0; k < n + 8; ++k) s += M[(size_t)k * n + i] * M[(size_t)k * n + j];
      h[(size_t)j * n + i] = s;
    }
  // io: [tile t (t = 0 diag, 1..4 below): element (r, c) at 256 t + 16 c + r] + zero at 1024
  std::vector<double> hio(1088, 0.0);
  for (int t = 0; t < 4; ++t)
    for (int c = 0; c < 16; ++c)
      for (int r = 0; r < 16; ++r) hio[256 * t + 16 * c + r] = h[(size_t)c * n + 16 * t + r];
  double *io, *out;
  unsigned long long* cyc;
  hipMalloc(&io, 1088 * 8);
  hipMalloc(&out, 1024 * 8);
  hipMalloc(&cyc, 8);
  hipMemcpy(io, hio.data(), 1088 * 8, hipMemcpyHostToDevice);
  std::vector<double> r0(1024), o(1024);
  auto run = [&](auto kern, const char* name, bool ref) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, io, out, cyc, 1);
    hipDeviceSynchronize();
    hipMemcpy(o.data(), out, 1024 * 8, hipMemcpyDeviceToHost);
    double md = 0.0;
    if (ref) r0 = o;
    else for (int i = 64; i < 64 + 768; ++i) md = std::max(md, std::abs(o[i] - r0[i]));
    std::vector<unsigned long long> cs;
    for (int rep = 0; rep < 5; ++rep) {
      hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, io, out, cyc, 400);
      hipDeviceSynchronize();
      unsigned long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      cs.push_back(c);
    }
    std::sort(cs.begin(), cs.end());
    printf("%-64s %6llu cycles per sweep (median of 5)  max|X - X_F0| %.1e\n", name, cs[2], md);
  };
  run(k_sweep<0>, "F0 shipped: 2 streams, v_fmac_f64_dpp", true);
  run(k_sweep<1>, "F1 2 streams, 2 x v_mov_b32_dpp broadcast + 2 v_fma_f64", false);
  run(k_sweep<2>, "F2 2 streams, readlane SGPR multiplier + 2 v_fma_f64", false);
  run(k_sweep<3>, "F3 1 stream (group 0 diag, 1-3 tiles), readlane multiplier + v_fma", false);
  run(k_sweep<4>, "F4 2 streams, v_mov_b64_dpp broadcast + 2 v_fma_f64", false);
  return 0;
}
