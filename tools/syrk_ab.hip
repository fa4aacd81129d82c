// Times the library's weighted KKT SYRK kernel (ipm_mfma.h, include path selects the version):
// H = C^T diag(w) C on n = 8192, m = 2048, lower triangle.  Diagnostic only.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#include "ipm_mfma.h"
int main() {
  const int n = 8192, m = 2048;
  double *X, *w, *C;
  hipMalloc(&X, (size_t)m * n * 8); hipMalloc(&w, m * 8); hipMalloc(&C, (size_t)n * n * 8);
  std::vector<double> h((size_t)m * n);
  for (size_t i = 0; i < h.size(); ++i) h[i] = (double)((i * 2654435761u) % 1000) / 1000.0 - 0.5;
  hipMemcpy(X, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  std::vector<double> hw(m, 0.7);
  hipMemcpy(w, hw.data(), m * 8, hipMemcpyHostToDevice);
  ipm::GemmArgs a;
  a.ni = a.nj = n; a.K = m; a.X = a.Y = X; a.ldx = a.ldy = n; a.w = w; a.C = C; a.ldc = n;
  a.alpha = 1.0; a.beta = 0.0; a.tri = 1;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  for (int r = 0; r < 3; ++r) ipm::mfma_gemm_launch(0, a);
  hipDeviceSynchronize();
  float best = 1e9, tot = 0;
  for (int r = 0; r < 10; ++r) {
    hipEventRecord(e0); ipm::mfma_gemm_launch(0, a); hipEventRecord(e1); hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1); best = ms < best ? ms : best; tot += ms;
  }
  printf("weighted SYRK n=%d m=%d: best %.3f ms avg %.3f ms  %.1f TF/s\n", n, m, best, tot / 10,
         (double)n * (n + 1) * m / best / 1e9);
  return 0;
}
