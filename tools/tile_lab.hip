// Trailing-tile lab (diagnostic only): the Cholesky's trailing update tile (C -= X^T Y, 128 x 128,
// K = 256, lower-triangle grid, C read first) as shipped vs. variants -- lazy C reads spread over
// the K loop, persistent workgroups.   scripts/chol_lab.sh runs it.
#define IPM_TILE_STAMPS 1
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../interiorpoint-gpu_amd/csrc/ipm_mfma.h"
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

template <bool LAZY, bool CST = false>
__global__ __launch_bounds__(256, 2) void k_tiles(ipm::GemmArgs a) {
  __shared__ ipm::MfSmem<128, 2> sm;
  for (int64_t L = blockIdx.x; L < a.nblk; L += gridDim.x)
    ipm::mfma_tile<128, false, true, 2, false, false, false, 1, LAZY, CST>(a, L, sm);
}

// phase-offset persistent tiles: the second workgroup to land on a CU waits g_delay ticks of the
// 100 MHz clock first, so that the two workgroups of a CU run half a tile apart (one's C traffic and
// prologue under the other's MFMAs)
__device__ unsigned g_cucnt[4096];
__device__ long long g_delay;
template <bool LAZY>
__global__ __launch_bounds__(256, 2) void k_tiles_phase(ipm::GemmArgs a) {
  __shared__ ipm::MfSmem<128, 2> sm;
  __shared__ int spar;
  if (threadIdx.x == 0) {
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    const unsigned key = ((xcc & 15u) << 8) | ((hw >> 8) & 0xFFu);
    spar = (int)(atomicAdd(&g_cucnt[key], 1u) & 1u);
  }
  __syncthreads();
  if (spar) {
    const long long t0 = __builtin_amdgcn_s_memrealtime();
    while ((long long)__builtin_amdgcn_s_memrealtime() - t0 < g_delay) __builtin_amdgcn_s_sleep(8);
  }
  for (int64_t L = blockIdx.x; L < a.nblk; L += gridDim.x)
    ipm::mfma_tile<128, false, true, 2, false, false, false, 1, LAZY>(a, L, sm);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 7680, reps = 10;
  const int KMAX = 2048;
  double *X, *C0, *C;
  CK(hipMalloc(&X, (size_t)KMAX * n * 8));
  CK(hipMalloc(&C0, (size_t)n * n * 8));
  CK(hipMalloc(&C, (size_t)n * n * 8));
  std::vector<double> h((size_t)std::max(KMAX, n) * n);
  srand(3);
  for (size_t i = 0; i < (size_t)KMAX * n; ++i) h[i] = rand() / (double)RAND_MAX - 0.5;
  CK(hipMemcpy(X, h.data(), (size_t)KMAX * n * 8, hipMemcpyHostToDevice));
  for (size_t i = 0; i < (size_t)n * n; ++i) h[i] = rand() / (double)RAND_MAX;
  CK(hipMemcpy(C0, h.data(), (size_t)n * n * 8, hipMemcpyHostToDevice));
  ipm::GemmArgs a;
  a.ni = a.nj = n; a.K = 256; a.X = a.Y = X; a.ldx = a.ldy = n; a.C = C; a.ldc = n; a.sub = 1; a.tri = 1;
  a.xcd_remap = 1; a.tiles_i = n / 128; a.nblk = a.tiles_i * (a.tiles_i + 1) / 2;
  std::vector<double> ref;
  auto run = [&](auto kern, const char* name, int grid, bool check) {
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    std::vector<float> t;
    for (int r = 0; r < reps; ++r) {
      CK(hipMemcpy(C, C0, (size_t)n * n * 8, hipMemcpyDeviceToDevice));
      CK(hipDeviceSynchronize());
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, a);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms; hipEventElapsedTime(&ms, e0, e1); t.push_back(ms);
    }
    std::sort(t.begin(), t.end());
    double d = 0;
    if (check) {
      std::vector<double> o((size_t)n * n);
      CK(hipMemcpy(o.data(), C, o.size() * 8, hipMemcpyDeviceToHost));
      if (ref.empty()) ref = o;
      else for (int j = 0; j < n; j += 7) for (int i = j; i < n; ++i) d = std::max(d, std::abs(o[(size_t)j * n + i] - ref[(size_t)j * n + i]));
    }
    const double fl = (double)n * (n + 1) * a.K, rounds = std::ceil((double)a.nblk / 512.0);
    printf("K=%4ld %-36s grid %5d  median %.3f ms  %.1f TF/s  %.1f us per tile (%.0f rounds), %.1f us per 256-K  max|dC| %.1e\n",
           (long)a.K, name, grid, t[t.size() / 2], fl / (t[t.size() / 2] * 1e-3) / 1e12, t[t.size() / 2] * 1e3 / rounds,
           rounds, t[t.size() / 2] * 1e3 / rounds * 256.0 / a.K, d);
  };
  auto stamps = [&](const char* name) {
    std::vector<unsigned long long> st(4096 * 8);
    CK(hipMemcpyFromSymbol(st.data(), HIP_SYMBOL(ipm::ipm_tile_stamps), st.size() * 8));
    const int nb = (int)std::min<int64_t>(a.nblk, 4096);
    unsigned long long r0 = ~0ull;
    for (int b = 0; b < nb; ++b) r0 = std::min(r0, st[b * 8 + 6]);
    printf("  stamps %s (cycles; per round of 512 workgroups by blockIdx):\n", name);
    for (int q = 0; q * 512 < nb; ++q) {
      double pro = 0, loop = 0, epi = 0, drain = 0, t0 = 0, t1 = 0; int c = 0;
      for (int b = q * 512; b < std::min(nb, q * 512 + 512); ++b, ++c) {
        const unsigned long long* x = &st[b * 8];
        pro += x[1] - x[0]; loop += x[2] - x[1]; epi += x[3] - x[2]; drain += x[4] - x[3];
        t0 += (x[6] - r0) / 100.0; t1 += (x[7] - r0) / 100.0;
      }
      printf("    blocks %4d-%4d: prologue %6.0f  slab loop %6.0f  epilogue issue %5.0f  store drain %5.0f | start %.1f us end %.1f us (means)\n",
             q * 512, q * 512 + c - 1, pro / c, loop / c, epi / c, drain / c, t0 / c, t1 / c);
    }
  };
  run(k_tiles<false>, "shipped (C read first)", (int)a.nblk, true);
  stamps("shipped K=256");
  run(k_tiles<true>, "lazy C (one block per slab)", (int)a.nblk, true);
  run(k_tiles<false>, "shipped, persistent 512 workgroups", 512, true);
  for (long long d : {0LL, 2000LL, 4000LL, 6000LL}) {   // ticks of 10 ns
    std::vector<unsigned> z(4096, 0u);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_delay), &d, sizeof(d)));
    char nm[96];
    snprintf(nm, sizeof nm, "phase offset %lld us, persistent 512", d / 100);
    // (the per-CU counters only need parity: they keep counting across repetitions, 2 per CU each)
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_cucnt), z.data(), z.size() * 4));
    run(k_tiles_phase<false>, nm, 512, true);
    CK(hipMemcpyToSymbol(HIP_SYMBOL(g_cucnt), z.data(), z.size() * 4));
    snprintf(nm, sizeof nm, "phase offset %lld us, persistent 512, lazy C", d / 100);
    run(k_tiles_phase<true>, nm, 512, true);
  }
  for (int K : {256, 512, 1024, 2048}) {
    a.K = K;
    a.sub = 1; a.alpha = 1.0; a.beta = 0.0;
    run(k_tiles<false>, "C -= X^T Y (C read + write)", (int)a.nblk, false);
    stamps("C -= X^T Y");
    a.sub = 0; a.alpha = -1.0; a.beta = 0.0;
    run(k_tiles<false>, "C = -X^T Y (write only)", (int)a.nblk, false);
    stamps("write only");
  }
  return 0;
}
