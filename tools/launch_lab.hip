// Host cost of a kernel launch and of a graph replay (diagnostic only, not part of the library).
#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
struct Big { double v[140]; };   // ~1.1 KB by-value argument, like BlockArgs
__global__ void k_empty(int* p) { if (threadIdx.x == 0 && p) p[blockIdx.x & 1] += 0; }
__global__ void k_big(Big b, int* p) { if (threadIdx.x == 0 && p) p[0] += (int)b.v[3]; }
int main() {
  hipStream_t st;
  hipStreamCreate(&st);
  int* p;
  hipMalloc(&p, 64);
  Big b{};
  auto now = [] { return std::chrono::steady_clock::now(); };
  for (int w = 0; w < 100; ++w) hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, p);
  hipStreamSynchronize(st);
  const int N = 2000;
  auto t0 = now();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_empty, dim3(8), dim3(256), 0, st, p);
  auto t1 = now();
  hipStreamSynchronize(st);
  auto t2 = now();
  printf("empty kernel: host %.2f us per launch, host+device %.2f us per launch\n",
         std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
         std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
  t0 = now();
  for (int i = 0; i < N; ++i) hipLaunchKernelGGL(k_big, dim3(8), dim3(256), 0, st, b, p);
  t1 = now();
  hipStreamSynchronize(st);
  t2 = now();
  printf("1.1 KB-arg kernel: host %.2f us per launch, host+device %.2f us per launch\n",
         std::chrono::duration<double, std::micro>(t1 - t0).count() / N,
         std::chrono::duration<double, std::micro>(t2 - t0).count() / N);
  // graph of 20 launches
  hipGraph_t g;
  hipGraphExec_t ge;
  hipStreamBeginCapture(st, hipStreamCaptureModeThreadLocal);
  for (int i = 0; i < 20; ++i) hipLaunchKernelGGL(k_big, dim3(8), dim3(256), 0, st, b, p);
  hipStreamEndCapture(st, &g);
  hipGraphInstantiate(&ge, g, nullptr, nullptr, 0);
  for (int w = 0; w < 10; ++w) hipGraphLaunch(ge, st);
  hipStreamSynchronize(st);
  const int R = 200;
  t0 = now();
  for (int i = 0; i < R; ++i) hipGraphLaunch(ge, st);
  t1 = now();
  hipStreamSynchronize(st);
  t2 = now();
  printf("graph of 20: host %.2f us per replay, host+device %.2f us per replay (%.2f per node)\n",
         std::chrono::duration<double, std::micro>(t1 - t0).count() / R,
         std::chrono::duration<double, std::micro>(t2 - t0).count() / R,
         std::chrono::duration<double, std::micro>(t2 - t0).count() / R / 20);
  // synchronize round trip
  t0 = now();
  for (int i = 0; i < 200; ++i) { hipLaunchKernelGGL(k_empty, dim3(1), dim3(64), 0, st, p); hipStreamSynchronize(st); }
  t1 = now();
  printf("launch + synchronize round trip %.2f us\n", std::chrono::duration<double, std::micro>(t1 - t0).count() / 200);
  return 0;
}
