// Does a busy GPU (trailing-update GEMM on other CUs) slow the single-workgroup Cholesky
// diagonal kernel?  Diagnostic only.
#define IPM_STAMPS 1
#include "../interiorpoint-gpu_amd/csrc/ipm_blas.hip"
#include <cstdio>
#include <vector>
#include <algorithm>
__global__ void k_probe(unsigned long long* out) {
  if (threadIdx.x == 0) {
    unsigned hw; asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
    unsigned xcc; asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc));
    out[blockIdx.x] = ((unsigned long long)xcc << 32) | hw;
  }
}
int main(int argc, char** argv) {
  const int mode = argc > 1 ? atoi(argv[1]) : 0;   // 0 alone, 1 concurrent no mask, 2 concurrent masked
  const int n = 8192, K = 256;
  double *X, *C, *A, *ws; int* info;
  hipMalloc(&X, (size_t)K * n * 8); hipMalloc(&C, (size_t)n * n * 8); hipMalloc(&A, 256 * 256 * 8);
  hipMalloc(&ws, 4096 * 8); hipMalloc(&info, 4);
  hipMemset(X, 0, (size_t)K * n * 8); hipMemset(C, 0, (size_t)n * n * 8);
  std::vector<double> h(256 * 256);
  for (int j = 0; j < 256; ++j) for (int i = 0; i < 256; ++i) h[j * 256 + i] = (i == j) ? 256.0 : 0.01 * ((i * 7 + j * 3) % 11 - 5);
  for (int j = 0; j < 256; ++j) for (int i = 0; i < j; ++i) h[j * 256 + i] = h[i * 256 + j];
  hipStream_t s1, s2;
  hipDeviceProp_t prop; hipGetDeviceProperties(&prop, 0);
  const int ncu = prop.multiProcessorCount;
  if (mode == 2) {
    std::vector<uint32_t> mm((ncu + 31) / 32, 0), ms((ncu + 31) / 32, 0);
    for (int i = 0; i < ncu; ++i) { if (i % 8 == 0) ms[i / 32] |= 1u << (i % 32); else mm[i / 32] |= 1u << (i % 32); }
    hipExtStreamCreateWithCUMask(&s1, mm.size(), mm.data());
    hipExtStreamCreateWithCUMask(&s2, ms.size(), ms.data());
  } else {
    hipStreamCreateWithFlags(&s1, hipStreamNonBlocking); hipStreamCreateWithFlags(&s2, hipStreamNonBlocking);
  }
  {
    unsigned long long* pr; hipMalloc(&pr, 4096 * 8);
    for (int which = 1; which <= 2; ++which) {
      hipLaunchKernelGGL(k_probe, dim3(2048), dim3(64), 0, which == 1 ? s1 : s2, pr);
      std::vector<unsigned long long> hp(2048);
      hipMemcpy(hp.data(), pr, 2048 * 8, hipMemcpyDeviceToHost);
      std::vector<int> seen;
      for (auto v : hp) {
        unsigned hw = (unsigned)v, xcc = (unsigned)(v >> 32);
        int cu = (hw >> 8) & 15, sh = (hw >> 12) & 1, se = (hw >> 13) & 7;
        int key = xcc * 1000 + se * 100 + sh * 16 + cu;
        if (std::find(seen.begin(), seen.end(), key) == seen.end()) seen.push_back(key);
      }
      std::sort(seen.begin(), seen.end());
      printf("stream %d: %zu distinct CUs:", which, seen.size());
      for (size_t i = 0; i < seen.size() && i < 40; ++i) printf(" %d", seen[i]);
      printf("\n");
    }
  }
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice); hipMemset(info, 0, 4);
    hipDeviceSynchronize();
    if (mode > 0) {
      ipm::GemmArgs a; a.ni = n; a.nj = n; a.K = K; a.X = X; a.ldx = n; a.Y = X; a.ldy = n; a.C = C; a.ldc = n; a.tri = 1;
      for (int r = 0; r < 4; ++r) ipm::mfma_gemm_launch(s1, a);
    }
    hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0, s2);
    hipLaunchKernelGGL(ipm::k_potrf_diag, dim3(1), dim3(256), 0, s2, (int64_t)0, 128, A, (int64_t)256, ws, info);
    hipEventRecord(e1, s2);
    hipEventSynchronize(e1);
    float ms; hipEventElapsedTime(&ms, e0, e1);
    unsigned long long st[64];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(ipm::ipm_stamps), sizeof(st));
    printf("mode %d rep %d: diag event %.1f us, in-kernel cycles %llu:", mode, rep, ms * 1e3, st[25] - st[0]); for (int i = 1; i < 26; ++i) printf(" %llu", st[i] - st[i - 1]); printf("\n");
    hipDeviceSynchronize();
  }
  return 0;
}
