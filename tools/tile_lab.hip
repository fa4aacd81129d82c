// Trailing-tile lab (diagnostic only): the Cholesky's trailing update tile (C -= X^T Y, 128 x 128,
// K = 256, lower-triangle grid, C read first) as shipped vs. variants -- lazy C reads spread over
// the K loop, persistent workgroups.   scripts/chol_lab.sh runs it.
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

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 7680, K = 256, reps = 10;
  double *X, *C0, *C;
  CK(hipMalloc(&X, (size_t)K * n * 8));
  CK(hipMalloc(&C0, (size_t)n * n * 8));
  CK(hipMalloc(&C, (size_t)n * n * 8));
  std::vector<double> h((size_t)std::max(K, n) * n);
  srand(3);
  for (size_t i = 0; i < (size_t)K * n; ++i) h[i] = rand() / (double)RAND_MAX - 0.5;
  CK(hipMemcpy(X, h.data(), (size_t)K * n * 8, hipMemcpyHostToDevice));
  for (size_t i = 0; i < (size_t)n * n; ++i) h[i] = rand() / (double)RAND_MAX;
  CK(hipMemcpy(C0, h.data(), (size_t)n * n * 8, hipMemcpyHostToDevice));
  ipm::GemmArgs a;
  a.ni = a.nj = n; a.K = K; a.X = a.Y = X; a.ldx = a.ldy = n; a.C = C; a.ldc = n; a.sub = 1; a.tri = 1;
  a.xcd_remap = 1; a.tiles_i = n / 128; a.nblk = a.tiles_i * (a.tiles_i + 1) / 2;
  std::vector<double> ref;
  auto run = [&](auto kern, const char* name, int grid) {
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
    std::vector<double> o((size_t)n * n);
    CK(hipMemcpy(o.data(), C, o.size() * 8, hipMemcpyDeviceToHost));
    double d = 0;
    if (ref.empty()) ref = o;
    else for (int j = 0; j < n; j += 7) for (int i = j; i < n; ++i) d = std::max(d, std::abs(o[(size_t)j * n + i] - ref[(size_t)j * n + i]));
    const double fl = (double)n * (n + 1) * K, rounds = (double)a.nblk / 512.0;
    printf("%-40s grid %5d  median %.3f ms  %.1f TF/s  %.1f us per 512-tile round  max|C - C_ref| %.1e\n", name, grid,
           t[t.size() / 2], fl / (t[t.size() / 2] * 1e-3) / 1e12, t[t.size() / 2] * 1e3 / rounds, d);
  };
  run(k_tiles<false>, "shipped (C read first)", (int)a.nblk);
  run(k_tiles<true>, "lazy C (one block per slab)", (int)a.nblk);
  run(k_tiles<false, true>, "C staged through LDS (1 KB columns)", (int)a.nblk);
  run(k_tiles<false>, "shipped (again)", (int)a.nblk);
  return 0;
}
