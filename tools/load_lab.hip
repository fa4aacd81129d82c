// How long does the Cholesky diagonal role take to bring its 128 x 128 lower block (36 blocks of
// 16 x 16, column-major, lda apart) into LDS?  One workgroup of 256 threads; s_memtime cycles from
// the first load to the barrier after the last.  Diagnostic only, never part of the library.
//   V0: global_load_lds 16 B per lane (the shipped path), aux 0      V1: same, aux 16 (sc1)
//   V2: agent-scope 8-byte atomic loads into registers, then LDS      V3: plain 16-byte loads
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

__device__ __forceinline__ int bidx(int I, int J) { return (I * (I + 1)) / 2 + J; }

template <int V>
__global__ __launch_bounds__(256, 1) void k_load(const double* A, long lda, long k0, unsigned long long* cyc,
                                                 double* out) {
  __shared__ double sD[36 * 256];
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  __syncthreads();
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  if (V <= 1) {
    int cnt = 0;
#pragma unroll
    for (int I = 0; I < 8; ++I)
#pragma unroll
      for (int J = 0; J <= I; ++J)
#pragma unroll
        for (int h = 0; h < 2; ++h, ++cnt)
          if ((cnt & 3) == wv) {
            const double* src = A + (k0 + J * 16 + (lane >> 3) + 8 * h) * lda + k0 + I * 16 + 2 * (lane & 7);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)&sD[bidx(I, J) * 256 + h * 128],
                                             16, 0, V == 1 ? 16 : 0);
          }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  } else if (V == 2) {
    // thread: element (r, c) of block q: 36 blocks x 256 elements / 256 threads = 36 per thread
    double v[36];
#pragma unroll
    for (int q = 0; q < 36; ++q) {
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= q) ++I;
      const int J = q - I * (I + 1) / 2;
      const int r = tid & 15, c = tid >> 4;
      const double* p = A + (k0 + J * 16 + c) * lda + k0 + I * 16 + r;
      v[q] = __longlong_as_double((long long)__hip_atomic_load(
          reinterpret_cast<unsigned long long*>(const_cast<double*>(p)), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
    }
#pragma unroll
    for (int q = 0; q < 36; ++q) sD[q * 256 + tid] = v[q];
  } else {
    double2 v[18];
#pragma unroll
    for (int q2 = 0; q2 < 18; ++q2) {
      const int q = 2 * q2 + (tid >> 7);
      int I = 0;
      while ((I + 1) * (I + 2) / 2 <= q) ++I;
      const int J = q - I * (I + 1) / 2;
      const int r2 = 2 * (tid & 7), c = (tid >> 3) & 15;
      v[q2] = *reinterpret_cast<const double2*>(A + (k0 + J * 16 + c) * lda + k0 + I * 16 + r2);
    }
#pragma unroll
    for (int q2 = 0; q2 < 18; ++q2) {
      const int q = 2 * q2 + (tid >> 7);
      const int r2 = 2 * (tid & 7), c = (tid >> 3) & 15;
      *reinterpret_cast<double2*>(&sD[q * 256 + c * 16 + r2]) = v[q2];
    }
  }
  __syncthreads();
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (tid == 0) cyc[0] = t1 - t0;
  double s = 0;
  for (int i = tid; i < 36 * 256; i += 256) s += sD[i];
  out[tid] = s;
}

// touch the block from many workgroups first (the fused kernel's loads follow other CUs' stores)
__global__ void k_touch(double* A, long lda, long k0) {
  const long j = k0 + blockIdx.x, i = k0 + threadIdx.x;
  A[j * lda + i] += 0.0 * (double)blockIdx.x + 1e-300;
}

int main() {
  const long n = 4096, lda = 4098, k0 = 1024;
  double *A, *out;
  unsigned long long* cyc;
  hipMalloc(&A, n * lda * 8);
  hipMalloc(&out, 256 * 8);
  hipMalloc(&cyc, 8);
  std::vector<double> h(n * lda, 1.0);
  hipMemcpy(A, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  auto run = [&](auto kern, const char* name) {
    for (int rep = 0; rep < 4; ++rep) {
      hipLaunchKernelGGL(k_touch, dim3(128), dim3(128), 0, 0, A, lda, k0);
      hipLaunchKernelGGL(kern, dim3(1), dim3(256), 0, 0, A, lda, k0, cyc, out);
      unsigned long long c;
      hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
      printf("%-44s rep %d: %6llu cycles\n", name, rep, c);
    }
  };
  run(k_load<0>, "global_load_lds 16B (shipped, aux 0)");
  run(k_load<1>, "global_load_lds 16B sc1 (shipped fused)");
  run(k_load<2>, "8-byte agent atomic loads -> LDS");
  run(k_load<3>, "plain 16-byte loads -> LDS");
  return 0;
}
