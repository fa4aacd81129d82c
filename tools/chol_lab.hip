// Cholesky diagonal-role lab (diagnostic only, never part of the library): times the fused
// diagonal role (ipm::diag_role<true, V>: the 128 x 128 diagonal block of a panel, one workgroup)
// in isolation for several variants V, on the same SPD block, and checks each variant's factor
// against variant 0 and against a host Cholesky.   Build + run: scripts/chol_lab.sh
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdio>
#include <vector>
#include <algorithm>
#include "../interiorpoint-gpu_amd/csrc/ipm_blas.hip"

template <int V>
__global__ __launch_bounds__(256, 2) void k_lab_diag(double* A, int64_t lda, double* ws, unsigned* ctl, int* info,
                                                     unsigned long long* cyc, int nb) {
  __shared__ ipm::DiagSmem sm;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  ipm::diag_role<true, V>(0, nb, A, lda, ws, info, ws + ipm::PF_DINV, &ctl[1], sm, &ctl[4]);
  __syncthreads();
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = t1 - t0;
}

static void host_chol(std::vector<double>& a, int n, int lda) {   // column-major lower, in place
  for (int j = 0; j < n; ++j) {
    double d = a[(size_t)j * lda + j];
    for (int k = 0; k < j; ++k) d -= a[(size_t)k * lda + j] * a[(size_t)k * lda + j];
    d = std::sqrt(d);
    a[(size_t)j * lda + j] = d;
    for (int i = j + 1; i < n; ++i) {
      double v = a[(size_t)j * lda + i];
      for (int k = 0; k < j; ++k) v -= a[(size_t)k * lda + i] * a[(size_t)k * lda + j];
      a[(size_t)j * lda + i] = v / d;
    }
  }
}

int main(int argc, char** argv) {
  const int nb = 128, lda = 128, reps = argc > 1 ? atoi(argv[1]) : 40;
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
  std::vector<double> ref = h;
  host_chol(ref, nb, lda);
  double *A0, *A, *ws;
  unsigned* ctl;
  int* info;
  unsigned long long* cyc;
  hipMalloc(&A0, h.size() * 8);
  hipMalloc(&A, h.size() * 8);
  hipMalloc(&ws, 32768 * 8);
  hipMalloc(&ctl, 64 * 4);
  hipMalloc(&info, 4);
  hipMalloc(&cyc, 8);
  hipMemcpy(A0, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  std::vector<double> out0;
  auto run = [&](auto kern, const char* name) {
    std::vector<double> cy, us;
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    for (int r = 0; r < reps; ++r) {
      hipMemcpy(A, A0, h.size() * 8, hipMemcpyDeviceToDevice);
      hipMemset(ctl, 0, 64 * 4);
      hipMemset(info, 0, 4);
      hipDeviceSynchronize();
      hipEventRecord(e0);
      hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, A, (int64_t)lda, ws, ctl, info, cyc, nb);
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      if (r >= 3) { cy.push_back((double)c); us.push_back(ms * 1e3); }
    }
    std::vector<double> o(h.size());
    hipMemcpy(o.data(), A, o.size() * 8, hipMemcpyDeviceToHost);
    int inf;
    hipMemcpy(&inf, info, 4, hipMemcpyDeviceToHost);
    double dref = 0, d0 = 0, nrm = 0;
    for (int j = 0; j < nb; ++j)
      for (int i = j; i < nb; ++i) {
        const size_t k = (size_t)j * lda + i;
        dref = std::max(dref, std::abs(o[k] - ref[k]));
        nrm = std::max(nrm, std::abs(ref[k]));
        if (!out0.empty()) d0 = std::max(d0, std::abs(o[k] - out0[k]));
      }
    if (out0.empty()) out0 = o;
    std::sort(cy.begin(), cy.end());
    std::sort(us.begin(), us.end());
    printf("%-44s median %7.0f cycles  min %7.0f  | event median %6.1f us | info %d | max|L-host|/max|L| %.1e  max|L-L_v0| %.1e\n",
           name, cy[cy.size() / 2], cy[0], us[us.size() / 2], inf, dref / nrm, d0);
  };
  run(k_lab_diag<130>, "V130 shipped (IPM_DIAG_V)");
  run(k_lab_diag<130 + 65536>, "V130 + lean leaf tail");
  run(k_lab_diag<130 + 65536 + 262144>, "V130 + lean tail + deferred write-back");
  run(k_lab_diag<130 + 65536 + 262144 + 524288>, "V130 + lean tail + deferred wb + deferred publish J>=2");
  run(k_lab_diag<130 + 65536 + 262144 + 1048576>, "V130 + lean tail + deferred wb + wave 3 tile at J<=2");
  run(k_lab_diag<130 + 65536 + 262144 + 524288 + 1048576>, "V130 + lean + dwb + dpub J>=2 + w3 tile");
  run(k_lab_diag<130 + 65536 + 8>, "V130 + lean tail + free waves idle (timing only)");
  run(k_lab_diag<130>, "V130 shipped (again)");
  return 0;
}
