// Where the diagonal role's time goes (diagnostic only): s_memtime phase stamps of
// ipm::diag_role<true, 2> on one 128 x 128 block, and the 16-column leaf sweep alone (one wave,
// registers only, repeated) in four forms.  Run: scripts/chol_lab.sh (second binary).
#define IPM_STAMPS 1
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../interiorpoint-gpu_amd/csrc/ipm_blas.hip"

template <int V>
__global__ __launch_bounds__(256, 2) void k_stamped(double* A, int64_t lda, double* ws, unsigned* ctl, int* info) {
  __shared__ ipm::DiagSmem sm;
  ipm::diag_role<true, V>(0, 128, A, lda, ws, info, ws + ipm::PF_DINV, &ctl[1], sm, &ctl[4]);
}

// M: 0 sweep as shipped (diag rows + tile-below rows), 1 diag rows only, 2 pivot chain only,
// 3 rank-1 DPP updates only (both row sets), 4 the restore step only (overhead)
template <int M>
__global__ __launch_bounds__(64) void k_sweep(const double* io, double* out, unsigned long long* cyc, int reps) {
  const int lane = threadIdx.x & 63, rr = lane & 15;
  const double zero = io[512];   // 0.0 at run time: the restore is exact (no denormal products)
  double orig[16], origb[16], row[16], rowb[16];
  for (int c = 0; c < 16; ++c) {
    orig[c] = io[c * 16 + rr];
    origb[c] = io[256 + c * 16 + rr];
    row[c] = orig[c];
    rowb[c] = origb[c];
  }
  double acc = 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < reps; ++it) {
    double piv = ipm::readlane_d(row[0], 0);
    double dv = ipm::rsqrt_pivot(piv);
    if (M != 4) {
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        acc += dv;
        double pivn = 1.0, dvn = 1.0;
        if (M != 3 && c + 1 < 16) {
          const double a1 = ipm::readlane_d(row[c], c + 1);
          const double d1 = ipm::readlane_d(row[c + 1], c + 1);
          const double l1 = a1 * dv;
          pivn = fma(-l1, l1, d1);
          dvn = ipm::rsqrt_pivot(pivn);
        }
        if (M != 2) {
          row[c] *= dv;
          if (M != 1) rowb[c] *= dv;
#pragma unroll
          for (int c2 = c + 1; c2 < 16; ++c2) {
            ipm::fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
            if (M != 1) ipm::fmac_bcast16(rowb[c2], row[c], rowb[c], c2, false);
          }
        }
        piv = pivn;
        if (M != 3) dv = dvn;
      }
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
}

// one register stream (diag_role V & 32768): group 0 diagonal rows, groups 1-3 tile rows, the
// multipliers through SGPRs (v_readlane); R: 0 = readlane per (c, c2), 1 = the column's multipliers
// read first, then the fmas
template <int R>
__global__ __launch_bounds__(64) void k_sweep_one(const double* io, double* out, unsigned long long* cyc, int reps) {
  const int lane = threadIdx.x & 63, rr = lane & 15, g = lane >> 4;
  const double zero = io[512];
  double orig[16], row[16];
  for (int c = 0; c < 16; ++c) {
    orig[c] = io[(g ? 256 : 0) + c * 16 + rr];
    row[c] = orig[c];
  }
  double acc = 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < reps; ++it) {
    double piv = ipm::readlane_d(row[0], 0);
    double dv = ipm::rsqrt_pivot(piv);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      acc += dv;
      double pivn = 1.0, dvn = 1.0;
      if (c + 1 < 16) {
        const double a1 = ipm::readlane_d(row[c], c + 1);
        const double d1 = ipm::readlane_d(row[c + 1], c + 1);
        const double l1 = a1 * dv;
        pivn = fma(-l1, l1, d1);
        dvn = ipm::rsqrt_pivot(pivn);
      }
      row[c] *= dv;
      if (R == 0) {
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) row[c2] = fma(-ipm::readlane_d(row[c], c2), row[c], row[c2]);
      } else {
        double m[16];
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) m[c2] = ipm::readlane_d(row[c], c2);
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) row[c2] = fma(-m[c2], row[c], row[c2]);
      }
      piv = pivn;
      dv = dvn;
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      acc += row[c];
      row[c] = fma(row[c], zero, orig[c]);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[0] = (t1 - t0) / reps;
  out[lane] = acc;
}

// the tile-below row update of the leaf in several forms (diag rows keep the shipped DPP fmac);
// F 0 shipped (v_fmac_f64_dpp rowb, -row_bcast, rowb), 1 readlane -> SGPR multiplier + v_fma,
// 2 asm v_mov_b64_dpp + v_fma, 3 builtin update_dpp + v_fma, 4 shipped with an s_nop 1 before every
// tile-row fmac, 5 shipped with the diag and tile-row loops split (all diag fmacs of column c
// first, then the tile-row fmacs)
__device__ __forceinline__ double movdpp(double x, int l) {
  double r;
  switch (l) {
#define C(k) case k: asm volatile("s_nop 1\n\tv_mov_b64_dpp %0, %1 row_newbcast:" #k " row_mask:0xf bank_mask:0xf" : "=v"(r) : "v"(x)); break;
    C(0) C(1) C(2) C(3) C(4) C(5) C(6) C(7) C(8) C(9) C(10) C(11) C(12) C(13) C(14) C(15)
#undef C
  }
  return r;
}
template <int F>
__global__ __launch_bounds__(64) void k_form(const double* io, double* out, unsigned long long* cyc, int reps) {
  const int lane = threadIdx.x & 63, rr = lane & 15;
  const double zero = io[512];
  double orig[16], origb[16], row[16], rowb[16];
  for (int c = 0; c < 16; ++c) {
    orig[c] = io[c * 16 + rr];
    origb[c] = io[256 + c * 16 + rr];
    row[c] = orig[c];
    rowb[c] = origb[c];
  }
  double acc = 0.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < reps; ++it) {
    double piv = ipm::readlane_d(row[0], 0);
    double dv = ipm::rsqrt_pivot(piv);
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      acc += dv;
      double pivn = 1.0, dvn = 1.0;
      if (c + 1 < 16) {
        const double a1 = ipm::readlane_d(row[c], c + 1);
        const double d1 = ipm::readlane_d(row[c + 1], c + 1);
        const double l1 = a1 * dv;
        pivn = fma(-l1, l1, d1);
        dvn = ipm::rsqrt_pivot(pivn);
      }
      row[c] *= dv;
      rowb[c] *= dv;
      if (F == 5) {
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) ipm::fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) ipm::fmac_bcast16(rowb[c2], row[c], rowb[c], c2, false);
      } else {
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) {
          ipm::fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
          if (F == 0) ipm::fmac_bcast16(rowb[c2], row[c], rowb[c], c2, false);
          if (F == 4) ipm::fmac_bcast16(rowb[c2], row[c], rowb[c], c2, true);
          if (F == 1) rowb[c2] = fma(-ipm::readlane_d(row[c], c2), rowb[c], rowb[c2]);
          if (F == 2) rowb[c2] = fma(-movdpp(row[c], c2), rowb[c], rowb[c2]);
          if (F == 3) rowb[c2] = fma(-ipm::bcast16(row[c], c2), rowb[c], rowb[c2]);
        }
      }
      piv = pivn;
      dv = dvn;
    }
#pragma unroll
    for (int c = 0; c < 16; ++c) {
      acc += row[c] + rowb[c];
      row[c] = fma(row[c], zero, orig[c]);
      rowb[c] = fma(rowb[c], zero, origb[c]);
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (lane == 0) cyc[0] = (t1 - t0) / reps;
  out[lane] = acc;
  if (reps == 1)
    for (int c = 0; c < 16; ++c) out[64 + c * 64 + lane] = rowb[c];
}

// the diag-only sweep in a 256-thread workgroup: W = 0 wave 0 sweeps, waves 1-3 wait at a barrier;
// W = 1 waves 0 and 1 sweep; W = 2 all four sweep (do waves of one workgroup share a SIMD?)
template <int W>
__global__ __launch_bounds__(256) void k_sweep4(const double* io, double* out, unsigned long long* cyc, int reps) {
  const int lane = threadIdx.x & 63, rr = lane & 15, wv = threadIdx.x >> 6;
  const double zero = io[512];
  double orig[16], row[16];
  for (int c = 0; c < 16; ++c) {
    orig[c] = io[c * 16 + rr];
    row[c] = orig[c];
  }
  double acc = 0.0;
  __syncthreads();
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  const bool active = wv == 0 || (W == 1 && wv == 1) || W == 2;
  if (active) {
    for (int it = 0; it < reps; ++it) {
      double piv = ipm::readlane_d(row[0], 0);
      double dv = ipm::rsqrt_pivot(piv);
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        acc += dv;
        double pivn = 1.0, dvn = 1.0;
        if (c + 1 < 16) {
          const double a1 = ipm::readlane_d(row[c], c + 1);
          const double d1 = ipm::readlane_d(row[c + 1], c + 1);
          const double l1 = a1 * dv;
          pivn = fma(-l1, l1, d1);
          dvn = ipm::rsqrt_pivot(pivn);
        }
        row[c] *= dv;
#pragma unroll
        for (int c2 = c + 1; c2 < 16; ++c2) ipm::fmac_bcast16(row[c2], row[c], row[c], c2, c2 == c + 1);
        piv = pivn;
        dv = dvn;
      }
#pragma unroll
      for (int c = 0; c < 16; ++c) {
        acc += row[c];
        row[c] = fma(row[c], zero, orig[c]);
      }
    }
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = (t1 - t0) / reps;
  __syncthreads();
  out[threadIdx.x] = acc;
}

int main() {
  const int nb = 128, lda = 128;
  std::vector<double> h((size_t)lda * nb);
  srand(7);
  std::vector<double> M((size_t)(nb + 8) * nb);
  for (auto& v : M) v = rand() / (double)RAND_MAX - 0.5;
  for (int j = 0; j < nb; ++j)
    for (int i = 0; i < nb; ++i) {
      double s = (i == j) ? 4.0 : 0.0;
      for (int k = 0; k < nb + 8; ++k) s += M[(size_t)k * nb + i] * M[(size_t)k * nb + j];
      h[(size_t)j * lda + i] = s;
    }
  double *A0, *A, *ws, *io, *out;
  unsigned* ctl;
  int* info;
  unsigned long long* cyc;
  hipMalloc(&A0, h.size() * 8); hipMalloc(&A, h.size() * 8); hipMalloc(&ws, 32768 * 8);
  hipMalloc(&ctl, 256); hipMalloc(&info, 4); hipMalloc(&cyc, 8); hipMalloc(&io, 520 * 8); hipMalloc(&out, 64 * 8);
  hipMemcpy(A0, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  auto stamped = [&](auto kern, int V) {
  for (int rep = 0; rep < 4; ++rep) {
    hipMemcpy(A, A0, h.size() * 8, hipMemcpyDeviceToDevice);
    hipMemset(ctl, 0, 256); hipMemset(info, 0, 4); hipDeviceSynchronize();
    hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, A, (int64_t)lda, ws, ctl, info);
    hipDeviceSynchronize();
    if (rep < 3) continue;
    unsigned long long s[128];
    hipMemcpyFromSymbol(s, HIP_SYMBOL(ipm::ipm_stamps), sizeof(s));
    printf("diag_role<true,%d> stamps (cycles): total %llu, panel load %llu\n", V, s[26] - s[0], s[1] - s[0]);
    if (V & 8192)
      for (int J = 0; J < 8; ++J)
        printf("  J=%d first (cold) sweep %lld, second (warm) sweep + stores %lld\n", J, (long long)(s[16 + J] - s[2 + 3 * J]),
               (long long)(s[32 + J] - s[16 + J]));
    printf("   leaf phases per J: step-1 barrier -> LDS operands landed / sweep alone / stores done:");
    for (int J = 0; J < 8; ++J)
      printf("  %lld/%lld/%lld", (long long)(s[48 + J] - s[2 + 3 * J]), (long long)(s[56 + J] - s[48 + J]),
             (long long)(s[32 + J] - s[56 + J]));
    printf("\n   J   step1+bar    leaf(w0)   bar-wait  progress   | inv(w3)  free-waves done (w1 w2 w3) from step1 end\n");
    for (int J = 0; J < 8; ++J) {
      const unsigned long long st = J == 0 ? s[1] : s[4 + 3 * (J - 1)];
      printf("  %2d  %9lld  %9lld  %9lld  %8lld   | %7lld  %7lld %7lld %7lld\n", J, (long long)(s[2 + 3 * J] - st),
             (long long)(s[32 + J] - s[2 + 3 * J]), (long long)(s[3 + 3 * J] - s[32 + J]),
             (long long)(s[4 + 3 * J] - s[3 + 3 * J]), J ? (long long)(s[40 + J] - s[2 + 3 * J]) : 0LL,
             J ? (long long)(s[80 + 8 + J] - s[2 + 3 * J]) : 0LL, J ? (long long)(s[80 + 16 + J] - s[2 + 3 * J]) : 0LL,
             J ? (long long)(s[80 + 24 + J] - s[2 + 3 * J]) : 0LL);
    }
  }
  };
  stamped(k_stamped<130 + 65536 + 262144 + 1048576>, 130 + 65536 + 262144 + 1048576);
  stamped(k_stamped<130 + 65536 + 262144 + 524288 + 1048576>, 130 + 65536 + 262144 + 524288 + 1048576);



  std::vector<double> hio(520, 0.0);
  for (int c = 0; c < 16; ++c)
    for (int r = 0; r < 16; ++r) {
      hio[c * 16 + r] = h[(size_t)c * lda + r];
      hio[256 + c * 16 + r] = h[(size_t)c * lda + 16 + r];
    }
  hipMemcpy(io, hio.data(), 520 * 8, hipMemcpyHostToDevice);
  auto sweep = [&](auto kern, const char* name) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, io, out, cyc, 200);
    hipDeviceSynchronize();
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-46s %6llu cycles per 16-column sweep (incl. restore)\n", name, c);
  };
  if (0) sweep(k_sweep<0>, "sweep as shipped (diag + tile-below rows)");
  if (0) sweep(k_sweep_one<0>, "one stream, readlane per fma");
  if (0) sweep(k_sweep_one<1>, "one stream, column multipliers first");
  sweep(k_sweep<1>, "diag rows only");
  sweep(k_sweep<2>, "pivot chain only");
  if (0) sweep(k_sweep<3>, "rank-1 DPP updates only (both row sets)");
  sweep(k_sweep<4>, "restore only");
  auto sweep4 = [&](auto kern, const char* name) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, io, out, cyc, 200);
    hipDeviceSynchronize();
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-46s %6llu cycles per 16-column sweep (incl. restore)\n", name, c);
  };
  hipMalloc(&out, 1088 * 8);
  sweep4(k_sweep4<0>, "diag rows only, 4-wave WG, wave 0 sweeps");
  sweep4(k_sweep4<1>, "diag rows only, 4-wave WG, waves 0+1 sweep");
  sweep4(k_sweep4<2>, "diag rows only, 4-wave WG, all 4 sweep");
  std::vector<double> r0(1088), r1(1088);
  auto form = [&](auto kern, const char* name, std::vector<double>* keep) {
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, io, out, cyc, 1);
    hipDeviceSynchronize();
    std::vector<double> o(1088);
    hipMemcpy(o.data(), out, 1088 * 8, hipMemcpyDeviceToHost);
    double md = 0;
    if (keep == nullptr) for (int i = 64; i < 1088; ++i) md = std::max(md, std::abs(o[i] - r0[i]));
    else *keep = o;
    hipLaunchKernelGGL(kern, dim3(1), dim3(64), 0, 0, io, out, cyc, 200);
    hipDeviceSynchronize();
    unsigned long long c;
    hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
    printf("%-46s %6llu cycles per sweep   max|X - X_F0| %.1e\n", name, c, md);
  };
  hipMalloc(&out, 1088 * 8);
  if (0) form(k_form<0>, "F0 tile rows: shipped DPP fmac", &r0);
  if (0) form(k_form<1>, "F1 tile rows: readlane multiplier + fma", nullptr);
  if (0) form(k_form<2>, "F2 tile rows: v_mov_b64_dpp + fma", nullptr);
  if (0) form(k_form<3>, "F3 tile rows: builtin update_dpp + fma", nullptr);
  if (0) form(k_form<4>, "F4 tile rows: DPP fmac with s_nop 1", nullptr);
  if (0) form(k_form<5>, "F5 tile rows: DPP fmac, loops split", nullptr);
  return 0;
}
