// Phase stamps of the Cholesky diagonal-block kernel (diagnostic build; never timed as a result).
#define IPM_STAMPS 1
#include "../interiorpoint-gpu_amd/csrc/ipm_blas.hip"
#include <cstdio>
#include <vector>
int main() {
  const int n = 256, lda = 256;
  std::vector<double> h((size_t)n * n);
  srand(3);
  for (int j = 0; j < n; ++j) for (int i = 0; i < n; ++i) h[(size_t)j * n + i] = (i == j) ? n : (rand() / (double)RAND_MAX - 0.5);
  for (int j = 0; j < n; ++j) for (int i = 0; i < j; ++i) h[(size_t)j * n + i] = h[(size_t)i * n + j];
  double *A, *ws; int* info;
  hipMalloc(&A, h.size() * 8); hipMalloc(&ws, 16384 * 8); hipMalloc(&info, 4);
  for (int rep = 0; rep < 3; ++rep) {
    hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice); hipMemset(info, 0, 4);
    hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
    hipEventRecord(a);
    hipMemset(ws + 2048 + 9216, 0, 64); hipLaunchKernelGGL(ipm::k_potrf_panel, dim3(1), dim3(256), 0, 0, (int64_t)128, (int64_t)0, 128, 0, A, (int64_t)lda, ws, (unsigned*)(ws + 2048 + 9216), info);
    hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b);
    unsigned long long st[128];
    hipMemcpyFromSymbol(st, HIP_SYMBOL(ipm::ipm_stamps), sizeof(st));
    printf("rep %d: %.1f us  load %llu cycles; per J: update / leaf+barrier / subst+barrier\n", rep, ms * 1e3,
           st[1] - st[0]);
    for (int J = 0; J < 8; ++J)
      printf("  J=%d  %5llu %5llu %5llu   leaf end %5llu  inv end %5lld  pub end %5lld (from update end)\n", J,
             st[2 + 3 * J] - st[1 + 3 * J], st[3 + 3 * J] - st[2 + 3 * J], st[4 + 3 * J] - st[3 + 3 * J],
             st[32 + J] - st[2 + 3 * J], J ? (long long)(st[40 + J] - st[2 + 3 * J]) : 0LL,
             J ? (long long)(st[48 + J] - st[2 + 3 * J]) : 0LL);
    printf("  tail %llu  total %llu\n", st[26] - st[25], st[26] - st[0]);
    for (int J = 1; J < 8; ++J)
      printf("  J=%d wave1: writeback done %6lld, updates done %6lld | wave2: publish done %6lld, updates done %6lld\n", J,
             (long long)(st[72 + J] - st[2 + 3 * J]), (long long)(st[88 + J] - st[2 + 3 * J]),
             (long long)(st[80 + J] - st[2 + 3 * J]), (long long)(st[96 + J] - st[2 + 3 * J]));
  }
  return 0;
}
