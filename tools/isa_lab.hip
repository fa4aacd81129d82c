// Issue cost of the fp64 instruction forms the Cholesky leaf can use (diagnostic only, never part
// of the library): one wave, 16 independent accumulators, each form repeated, s_memtime per
// instruction.  Build + run on the GPU box:  hipcc --offload-arch=gfx950 -O3 tools/isa_lab.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define R16(X) X(0) X(1) X(2) X(3) X(4) X(5) X(6) X(7) X(8) X(9) X(10) X(11) X(12) X(13) X(14) X(15)

template <int F>
__global__ __launch_bounds__(64) void k_form(double* out, unsigned long long* cyc, int reps, double seed) {
  double a0 = seed, a1 = seed + 1, a2 = seed + 2, a3 = seed + 3, a4 = seed + 4, a5 = seed + 5, a6 = seed + 6,
         a7 = seed + 7, a8 = seed + 8, a9 = seed + 9, a10 = seed + 10, a11 = seed + 11, a12 = seed + 12,
         a13 = seed + 13, a14 = seed + 14, a15 = seed + 15;
  double x = seed * 0.5 + threadIdx.x, y = seed * 0.25;
  const double s = __builtin_amdgcn_readfirstlane((int)seed) * 1.0;
  unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < reps; ++it) {
#define ACC(k) a##k
    if constexpr (F == 0) {   // v_fmac_f64_dpp row_newbcast (the shipped leaf update)
#define X(k) asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(ACC(k)) : "v"(x), "v"(y));
      R16(X)
#undef X
    } else if constexpr (F == 1) {   // plain v_fma_f64 (vector operands)
#define X(k) asm volatile("v_fma_f64 %0, -%1, %2, %0" : "+v"(ACC(k)) : "v"(x), "v"(y));
      R16(X)
#undef X
    } else if constexpr (F == 2) {   // v_fma_f64 with an SGPR-pair operand
#define X(k) asm volatile("v_fma_f64 %0, -%1, %2, %0" : "+v"(ACC(k)) : "s"(s), "v"(y));
      R16(X)
#undef X
    } else if constexpr (F == 3) {   // v_mov_b64_dpp row_newbcast
#define X(k) asm volatile("v_mov_b64_dpp %0, %1 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "=v"(ACC(k)) : "v"(x));
      R16(X)
#undef X
    } else if constexpr (F == 4) {   // v_readlane_b32 (x2 per double)
#define X(k) { int lo, hi; asm volatile("v_readlane_b32 %0, %2, 3\n\tv_readlane_b32 %1, %3, 3" : "=s"(lo), "=s"(hi) : "v"(__double2loint(x)), "v"(__double2hiint(x))); ACC(k) += __hiloint2double(hi, lo); }
      R16(X)
#undef X
    } else if constexpr (F == 5) {   // v_mov_b32_dpp row_newbcast x2 per double
#define X(k) { int lo, hi; asm volatile("v_mov_b32_dpp %0, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_mov_b32_dpp %1, %3 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "=v"(lo), "=v"(hi) : "v"(__double2loint(x)), "v"(__double2hiint(x))); ACC(k) += __hiloint2double(hi, lo); }
      R16(X)
#undef X
    } else if constexpr (F == 6) {   // dependent chain of v_fma_f64 (latency)
#define X(k) asm volatile("v_fma_f64 %0, -%1, %2, %0" : "+v"(a0) : "v"(x), "v"(y));
      R16(X)
#undef X
    } else if constexpr (F == 7) {   // dependent chain of v_fmac_f64_dpp (latency)
#define X(k) asm volatile("v_fmac_f64_dpp %0, -%1, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf" : "+v"(a0) : "v"(x), "v"(y));
      R16(X)
#undef X
    } else if constexpr (F == 8) {   // v_mul_f64
#define X(k) asm volatile("v_mul_f64 %0, %1, %0" : "+v"(ACC(k)) : "v"(y));
      R16(X)
#undef X
    } else if constexpr (F == 9) {   // v_fmac_f64_e32 (VOP2, no DPP)
#define X(k) asm volatile("v_fmac_f64_e32 %0, %1, %2" : "+v"(ACC(k)) : "v"(x), "v"(y));
      R16(X)
#undef X
    } else if constexpr (F == 10) {   // v_rsq_f64
#define X(k) asm volatile("v_rsq_f64 %0, %1" : "=v"(ACC(k)) : "v"(y));
      R16(X)
#undef X
    } else if constexpr (F == 11) {   // v_pk_fma_f32-free control: s_nop 0
#define X(k) asm volatile("s_nop 0");
      R16(X)
#undef X
    }
#undef ACC
  }
  unsigned long long t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) cyc[0] = (t1 - t0);
  out[threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + a8 + a9 + a10 + a11 + a12 + a13 + a14 + a15;
}

template <int F>
static void run(const char* name, double* out, unsigned long long* cyc) {
  const int reps = 4096;
  hipLaunchKernelGGL((k_form<F>), dim3(1), dim3(64), 0, 0, out, cyc, 16, 1.0);   // warm
  hipDeviceSynchronize();
  hipLaunchKernelGGL((k_form<F>), dim3(1), dim3(64), 0, 0, out, cyc, reps, 1.0);
  hipDeviceSynchronize();
  unsigned long long c;
  hipMemcpy(&c, cyc, 8, hipMemcpyDeviceToHost);
  printf("%-44s %6.2f cycles per instruction\n", name, (double)c / (reps * 16.0));
}

int main() {
  double* out;
  unsigned long long* cyc;
  hipMalloc(&out, 64 * 8);
  hipMalloc(&cyc, 8);
  run<0>("v_fmac_f64_dpp row_newbcast (indep)", out, cyc);
  run<1>("v_fma_f64 vector operands (indep)", out, cyc);
  run<2>("v_fma_f64 SGPR-pair operand (indep)", out, cyc);
  run<3>("v_mov_b64_dpp row_newbcast (indep)", out, cyc);
  run<4>("2 x v_readlane_b32 + v_add_f64", out, cyc);
  run<5>("2 x v_mov_b32_dpp + v_add_f64", out, cyc);
  run<6>("v_fma_f64 dependent chain", out, cyc);
  run<7>("v_fmac_f64_dpp dependent chain", out, cyc);
  run<8>("v_mul_f64 (indep)", out, cyc);
  run<9>("v_fmac_f64_e32 (indep)", out, cyc);
  run<10>("v_rsq_f64 (indep)", out, cyc);
  run<11>("s_nop 0", out, cyc);
  return 0;
}
