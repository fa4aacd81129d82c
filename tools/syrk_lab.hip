// KKT SYRK lab (diagnostic only): the library's launch (mfma_gemm_launch_split: stream-K or
// K-halves tail, IPM_STREAMK picks the mode) on H = C^T diag(w) C + tP P + diag(d), lower
// triangle, with per-workgroup entry / exit stamps (100 MHz clock), against the same tile on a
// full square grid.   tools/syrk_lab N K [reps]
#define IPM_TILE_STAMPS 1
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include "../interiorpoint-gpu_amd/csrc/ipm_mfma.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

__device__ unsigned long long g_now[4];
__global__ void k_now(int i) { g_now[i] = __builtin_amdgcn_s_memrealtime(); }

static int ncu() {
  int d = 0, c = 0;
  hipGetDevice(&d);
  hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, d);
  return c;
}

int main(int argc, char** argv) {
  const int64_t n = argc > 1 ? atol(argv[1]) : 8192, K = argc > 2 ? atol(argv[2]) : 2048;
  const int reps = argc > 3 ? atoi(argv[3]) : 10;
  const int64_t ldx = n, ldc = (n + 15) / 16 * 16;
  double *X, *w, *P, *dv, *C, *ws;
  CK(hipMalloc(&X, (size_t)K * ldx * 8));
  CK(hipMalloc(&w, (size_t)K * 8));
  CK(hipMalloc(&P, (size_t)n * n * 8));
  CK(hipMalloc(&dv, (size_t)n * 8));
  CK(hipMalloc(&C, (size_t)n * ldc * 8));
  const int slots = 2 * ncu();
  const int64_t cap = 512;   // partial tiles (the engine's syrk_split_cap order of magnitude)
  CK(hipMalloc(&ws, (size_t)cap * 128 * 128 * 8 + (size_t)(2 * cap + 4096) * 4));
  CK(hipMemset(ws, 0, (size_t)cap * 128 * 128 * 8 + (size_t)(2 * cap + 4096) * 4));
  {
    std::vector<double> h((size_t)K * ldx);
    srand(5);
    for (auto& v : h) v = rand() / (double)RAND_MAX - 0.5;
    CK(hipMemcpy(X, h.data(), h.size() * 8, hipMemcpyHostToDevice));
    std::vector<double> hw(K);
    for (auto& v : hw) v = 0.5 + rand() / (double)RAND_MAX;
    CK(hipMemcpy(w, hw.data(), K * 8, hipMemcpyHostToDevice));
    std::vector<double> hp((size_t)n * n, 0.0);
    for (int64_t i = 0; i < n; ++i) hp[i * n + i] = 1.0;
    CK(hipMemcpy(P, hp.data(), hp.size() * 8, hipMemcpyHostToDevice));
    CK(hipMemcpy(dv, hw.data(), std::min<int64_t>(n, K) * 8, hipMemcpyHostToDevice));
  }
  ipm::GemmArgs a;
  a.ni = a.nj = n; a.K = K; a.X = a.Y = X; a.ldx = a.ldy = ldx; a.w = w; a.C = C; a.ldc = ldc;
  a.alpha = 1.0; a.beta = 0.0; a.P = P; a.ldp = n; a.tP = 0.5; a.dvec = dv; a.tri = 1;
  hipEvent_t e0, e1;
  hipEventCreate(&e0); hipEventCreate(&e1);
  auto timeit = [&](auto fn) {
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
      hipEventRecord(e0);
      fn();
      hipEventRecord(e1);
      CK(hipEventSynchronize(e1));
      float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    return t[t.size() / 2];
  };
  const double fl = (double)n * (n + 1) * K;
  const int64_t T = (n + 127) / 128, ntri = T * (T + 1) / 2;
  const char* mode = getenv("IPM_STREAMK");
  const float tlib = timeit([&] {
    hipLaunchKernelGGL(k_now, dim3(1), dim3(64), 0, 0, 0);
    ipm::mfma_gemm_launch_split(0, a, ws, cap, slots, false);
    hipLaunchKernelGGL(k_now, dim3(1), dim3(64), 0, 0, 1);
  });
  unsigned long long gn[4];
  CK(hipMemcpyFromSymbol(gn, HIP_SYMBOL(g_now), sizeof gn));
  printf("n=%ld K=%ld tiles=%ld slots=%d IPM_STREAMK=%s  library SYRK median %.3f ms  %.1f TF/s\n", (long)n,
         (long)K, (long)ntri, slots, mode ? mode : "(default)", tlib, fl / tlib / 1e9);
  // stamps of the last repetition: [6] entry, [7] exit (100 MHz), [1]/[2] slab loop (cycles)
  std::vector<unsigned long long> st(4096 * 8);
  CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(ipm::ipm_tile_stamps), st.size() * 8));
  int64_t qk = 0, Kp = 0;
  const int Pp = ipm::streamk_plan(ntri, slots, cap, K, qk, Kp);
  const int64_t s_full = ntri - qk, npc = qk * Pp;
  const int pl = ipm::streamk_mode(ntri, slots) == 2 ? 1 : 0;
  const int64_t nb = std::min<int64_t>(Pp ? s_full + npc : ntri, 4096);
  printf("  plan: P=%d Kp=%ld q=%ld whole=%ld pieces=%ld pieces_%s\n", Pp, (long)Kp, (long)qk, (long)s_full,
         (long)npc, pl ? "last" : "first");
  unsigned long long r0 = ~0ull, r1 = 0;
  for (int64_t b = 0; b < nb; ++b) { r0 = std::min(r0, st[b * 8 + 6]); r1 = std::max(r1, st[b * 8 + 7]); }
  printf("  stamped span %.1f us (first entry -> last exit); marker kernel before -> first entry %.1f us, last exit -> marker after %.1f us\n",
         (r1 - r0) / 100.0, ((double)r0 - (double)gn[0]) / 100.0, ((double)gn[1] - (double)r1) / 100.0);
  {   // per XCC: tile duration, slab-loop clock (s_memtime cycles over the 100 MHz duration)
    double dsum[8] = {0}, csum[8] = {0}, dmax[8] = {0}, dmin[8];
    int cnt[8] = {0};
    for (int x = 0; x < 8; ++x) dmin[x] = 1e30;
    for (int64_t b = 0; b < nb; ++b) {
      const unsigned long long* s = &st[b * 8];
      const int x = (int)((s[5] >> 32) & 7);
      const double d = (s[7] - s[6]) / 100.0;
      dsum[x] += d; dmax[x] = std::max(dmax[x], d); dmin[x] = std::min(dmin[x], d);
      csum[x] += (double)(s[4] - s[0]) / d;   // cycles per us of the whole tile
      ++cnt[x];
    }
    for (int x = 0; x < 8; ++x)
      if (cnt[x])
        printf("    xcc %d: %4d tiles  dur mean %7.1f min %7.1f max %7.1f us  s_memtime rate %.0f MHz\n", x, cnt[x],
               dsum[x] / cnt[x], dmin[x], dmax[x], csum[x] / cnt[x]);
    const char* dump = getenv("SYRK_LAB_DUMP");
    if (dump) {
      FILE* f = fopen(dump, "wb");
      if (f) { fwrite(st.data(), 8, (size_t)nb * 8, f); fclose(f); }
    }
  }
  auto cls = [&](int64_t b) {   // 0 whole, 1 piece
    if (!Pp) return 0;
    return pl ? (b < s_full ? 0 : 1) : (b < npc ? 1 : 0);
  };
  for (int c = 0; c < 2; ++c) {
    std::vector<double> s0, s1, d;
    for (int64_t b = 0; b < nb; ++b) {
      if (cls(b) != c) continue;
      s0.push_back((st[b * 8 + 6] - r0) / 100.0);
      s1.push_back((st[b * 8 + 7] - r0) / 100.0);
      d.push_back((st[b * 8 + 7] - st[b * 8 + 6]) / 100.0);
    }
    if (d.empty()) continue;
    auto mm = [](std::vector<double> v) { std::sort(v.begin(), v.end()); return v; };
    auto a0 = mm(s0), a1 = mm(s1), ad = mm(d);
    double mean = 0; for (double x : d) mean += x; mean /= d.size();
    printf("  %s n=%zu start %.1f..%.1f  end %.1f..%.1f (p50 %.1f p90 %.1f)  dur mean %.1f min %.1f p50 %.1f max %.1f\n",
           c ? "pieces" : "whole ", d.size(), a0.front(), a0.back(), a1.front(), a1.back(), a1[a1.size() / 2],
           a1[a1.size() * 9 / 10], mean, ad.front(), ad[ad.size() / 2], ad.back());
    if (c == 0) {   // whole tiles by start-time bucket
      const double bw = std::max(20.0, a1.back() / 12.0);
      for (double t = 0; t < a0.back() + bw; t += bw) {
        int cnt = 0; double dm = 0, em = 0;
        for (size_t i = 0; i < s0.size(); ++i)
          if (s0[i] >= t && s0[i] < t + bw) { ++cnt; dm += d[i]; em = std::max(em, s1[i]); }
        if (cnt) printf("    whole tiles starting %6.1f-%6.1f us: n=%4d dur mean %6.1f  last end %6.1f\n", t, t + bw, cnt, dm / cnt, em);
      }
    }
  }
  // the same tile on a full square grid, same K (no tail: T^2 tiles), and the plain triangle
  a.tri = 0; a.P = nullptr; a.dvec = nullptr;
  const float tfull = timeit([&] { ipm::mfma_gemm_launch_bm<128>(0, a, true); });
  printf("  full %ldx%ld grid, same tile: %.3f ms %.1f TF/s (%.1f rounds of %d)\n", (long)T, (long)T, tfull,
         2.0 * n * n * K / tfull / 1e9, (double)(T * T) / slots, slots);
  a.tri = 1;
  const float ttri = timeit([&] { ipm::mfma_gemm_launch_bm<128>(0, a, true); });
  printf("  plain triangle (no tail split, no epilogue): %.3f ms %.1f TF/s\n", ttri, fl / ttri / 1e9);
  return 0;
}
