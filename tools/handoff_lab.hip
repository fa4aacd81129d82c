// Cross-workgroup hand-off latency lab (diagnostic only): a chain of NSTEP workgroups, each waiting
// for its predecessor's value and then publishing its own (what the backward solve and the
// Cholesky's critical roles do per step), with the producer and consumer on different XCDs
// (consecutive blockIdx) or on the same XCD (blockIdx spaced by 8: blocks b, b+8, ... share an XCD,
// tools/syrk_lab.hip stamps), and with
//   mode 0: agent-scope relaxed atomics (global_store / global_load ... sc1: the library's protocol)
//   mode 1: plain store + L1-bypassing load (global_load ... sc0): coherent only inside one XCD
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/handoff_lab.hip -o build/r6lab/handoff_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr unsigned long long PEND = ~0ull;

__device__ __forceinline__ unsigned long long ld_mode(const unsigned long long* p, int mode) {
  if (mode == 0) return __hip_atomic_load(const_cast<unsigned long long*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  unsigned long long v;
  asm volatile("global_load_dwordx2 %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" : "=v"(v) : "v"(p) : "memory");
  return v;
}
__device__ __forceinline__ void st_mode(unsigned long long* p, unsigned long long v, int mode) {
  if (mode == 0) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else asm volatile("global_store_dwordx2 %0, %1, off sc0\n\ts_waitcnt vmcnt(0)" :: "v"(p), "v"(v) : "memory");
}

// y[k] for k < nstep: PEND before the run; step k = blockIdx / S (only blocks with blockIdx % S == 0 work)
__global__ __launch_bounds__(64) void k_chain(int nstep, int S, int mode, unsigned long long* y,
                                              unsigned long long* tstamp, unsigned* xcc, unsigned* err) {
  const int b = blockIdx.x;
  if (b % S != 0) return;
  const int k = b / S;
  if (k >= nstep) return;
  if (threadIdx.x == 0) xcc[k] = __builtin_amdgcn_s_getreg((31 << 11) | 20);
  unsigned long long prev = 0;
  if (k > 0) {
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      prev = ld_mode(&y[k - 1], mode);
      if (prev != PEND) break;
      __builtin_amdgcn_s_sleep(1);
      if (__builtin_amdgcn_s_memrealtime() - t0 > 100000000ull) {   // 1 s: give up, flag it
        if (threadIdx.x == 0) atomicOr(err, 1u);
        return;
      }
    }
  } else {
    if (threadIdx.x == 0) tstamp[0] = __builtin_amdgcn_s_memrealtime();
  }
  if (threadIdx.x == 0) {
    st_mode(&y[k], prev + 1, mode);
    if (k == nstep - 1) tstamp[1] = __builtin_amdgcn_s_memrealtime();
  }
}

int main(int argc, char** argv) {
  const int nstep = argc > 1 ? atoi(argv[1]) : 64;
  unsigned long long *y, *ts;
  unsigned *xcc, *err;
  CK(hipMalloc(&y, nstep * 8));
  CK(hipMalloc(&ts, 16));
  CK(hipMalloc(&xcc, nstep * 4));
  CK(hipMalloc(&err, 4));
  std::vector<unsigned long long> hy(nstep);
  std::vector<unsigned> hx(nstep);
  for (int mode = 0; mode < 2; ++mode)
    for (int S : {1, 8, 16}) {
      std::vector<double> per;
      bool ok = true, same = true;
      for (int rep = 0; rep < 12; ++rep) {
        CK(hipMemset(y, 0xFF, nstep * 8));
        CK(hipMemset(err, 0, 4));
        CK(hipDeviceSynchronize());
        hipLaunchKernelGGL(k_chain, dim3(nstep * S), dim3(64), 0, 0, nstep, S, mode, y, ts, xcc, err);
        CK(hipDeviceSynchronize());
        unsigned long long t[2];
        unsigned ev;
        CK(hipMemcpy(t, ts, 16, hipMemcpyDeviceToHost));
        CK(hipMemcpy(&ev, err, 4, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hy.data(), y, nstep * 8, hipMemcpyDeviceToHost));
        CK(hipMemcpy(hx.data(), xcc, nstep * 4, hipMemcpyDeviceToHost));
        if (ev || hy[nstep - 1] != (unsigned long long)nstep) ok = false;   // (step k stores k + 1)
        for (int k = 1; k < nstep; ++k) same = same && ((hx[k] & 7) == (hx[0] & 7));
        if (rep >= 2) per.push_back((t[1] - t[0]) / 100.0 / (nstep - 1));
      }
      std::sort(per.begin(), per.end());
      printf("mode %d (%s)  spacing %2d (%s XCD)  per hand-off: median %.2f us  min %.2f  max %.2f  %s\n", mode,
             mode ? "plain store + sc0 load" : "agent-scope sc1", S, same ? "same" : "changing", per[per.size() / 2],
             per.front(), per.back(), ok ? "ok" : "FAILED (wrong value or timeout)");
      fflush(stdout);
    }
  return 0;
}
