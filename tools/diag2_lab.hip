// Diagonal-role lab, round 4 (diagnostic only, never part of the library): the round-3 role
// (ipm::diag_role<true, 130>) against diag_role2 (ipm_diag2.h) on the same 128 x 128 SPD block:
// factor vs a host Cholesky, Dinv_J = L_JJ^-1 vs the host inverse, the final progress word, and
// the time of one role (s_memtime cycles, HIP events).  With -DIPM_STAMPS2 it also prints the
// per-step phase stamps of diag_role2.   Build + run: scripts/diag2_lab.sh
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <vector>
#include "../interiorpoint-gpu_amd/csrc/ipm_blas.hip"
namespace ipm {
#include "ipm_diag2.h"   // lab-only: not part of the library kernel
}

template <int ROLE>
__global__ __launch_bounds__(256, 2) void k_lab(double* A, int64_t lda, double* ws, unsigned* ctl, int* info,
                                                unsigned long long* cyc) {
  __shared__ union { ipm::DiagSmem d; ipm::Diag2Smem d2; } sm;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (ROLE == 0) ipm::diag_role<true, 130>(0, 128, A, lda, ws, info, ws + ipm::PF_DINV, &ctl[1], sm.d, &ctl[4]);
  else if (ROLE == 1) ipm::diag_role2<true, 0>(0, 128, A, lda, ws, info, ws + ipm::PF_DINV, &ctl[1], sm.d2, &ctl[4]);
  else ipm::diag_role2<true, 1>(0, 128, A, lda, ws, info, ws + ipm::PF_DINV, &ctl[1], sm.d2, &ctl[4]);
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
  const int nb = 128, lda = 130, reps = argc > 1 ? atoi(argv[1]) : 40;
  std::vector<double> h((size_t)lda * nb, 0.0);
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
  // host inverses of the eight 16 x 16 diagonal blocks of L
  std::vector<double> dref(8 * 256);
  for (int J = 0; J < 8; ++J)
    for (int c = 0; c < 16; ++c)
      for (int r = 0; r < 16; ++r) {   // X = L^-1: L X = I, column c by forward substitution
        double v = (r == c) ? 1.0 : 0.0;
        for (int k = c; k < r; ++k) v -= ref[(size_t)(J * 16 + k) * lda + J * 16 + r] * dref[J * 256 + c * 16 + k];
        dref[J * 256 + c * 16 + r] = v / ref[(size_t)(J * 16 + r) * lda + J * 16 + r];
      }
  double *A, *ws;
  unsigned* ctl;
  int* info;
  unsigned long long* cyc;
  hipMalloc(&A, h.size() * 8);
  hipMalloc(&ws, 32768 * 8);
  hipMalloc(&ctl, 64 * 4);
  hipMalloc(&info, 4);
  hipMalloc(&cyc, 8);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  auto run = [&](auto kern, const char* name) {
    std::vector<double> cy, us;
    for (int r = 0; r < reps; ++r) {
      hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
      hipMemset(ctl, 0, 64 * 4);
      hipMemset(info, 0, 4);
      hipMemset(ws, 0, 32768 * 8);
      hipEventRecord(e0, 0);
      hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, A, (int64_t)lda, ws, ctl, info, cyc);
      hipEventRecord(e1, 0);
      hipDeviceSynchronize();
      float ms;
      hipEventElapsedTime(&ms, e0, e1);
      unsigned long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      if (r >= 3) { cy.push_back((double)c); us.push_back(ms * 1e3); }
    }
    std::vector<double> o(h.size()), dv(8 * 256);
    hipMemcpy(o.data(), A, o.size() * 8, hipMemcpyDeviceToHost);
    hipMemcpy(dv.data(), ws, dv.size() * 8, hipMemcpyDeviceToHost);
    int inf;
    unsigned prog;
    hipMemcpy(&inf, info, 4, hipMemcpyDeviceToHost);
    hipMemcpy(&prog, ctl + 1, 4, hipMemcpyDeviceToHost);
    double el = 0, nrm = 0, ed = 0, nd = 0;
    for (int j = 0; j < nb; ++j)
      for (int i = j; i < nb; ++i) {
        const size_t k = (size_t)j * lda + i;
        el = std::max(el, std::abs(o[k] - ref[k]));
        nrm = std::max(nrm, std::abs(ref[k]));
      }
    for (int e = 0; e < 8 * 256; ++e) {
      ed = std::max(ed, std::abs(dv[e] - dref[e]));
      nd = std::max(nd, std::abs(dref[e]));
    }
    std::sort(cy.begin(), cy.end());
    std::sort(us.begin(), us.end());
    printf("%-34s median %7.0f cycles  min %7.0f | event median %6.1f us | info %d progress %u | L rel %.1e  Dinv rel %.1e\n",
           name, cy[cy.size() / 2], cy[0], us[us.size() / 2], inf, prog, el / nrm, ed / nd);
  };
  run(k_lab<0>, "diag_role<true,130> (round 3)");
#ifndef STAMP_V
  run(k_lab<1>, "diag_role2<0> (two leaf waves)");
#endif
  run(k_lab<2>, "diag_role2<1> (one leaf wave)");
  run(k_lab<0>, "diag_role<true,130> (again)");
#ifndef STAMP_V
  run(k_lab<1>, "diag_role2<0> (again)");
#endif
  run(k_lab<2>, "diag_role2<1> (again)");
#ifdef IPM_STAMPS2
  unsigned long long st[4][8][8];
  hipMemcpyFromSymbol(st, HIP_SYMBOL(ipm::ipm_stamps2), sizeof(st));
  const unsigned long long base = st[0][0][0];
  printf("diag_role2 stamps (cycles from wave 0's step-0 start): per step J, wave: start / after sweep-or-publish / end of A / after B1 / after B\n");
  for (int J = 0; J < 8; ++J) {
    printf("J=%d", J);
    for (int w = 0; w < 4; ++w)
      printf(" | w%d %6lld %6lld %6lld %6lld %6lld", w, (long long)(st[w][J][0] - base), (long long)(st[w][J][1] - base),
             (long long)(st[w][J][2] - base), (long long)(st[w][J][3] - base), (long long)(st[w][J][4] - base));
    printf("\n");
  }
#endif
  return 0;
}
