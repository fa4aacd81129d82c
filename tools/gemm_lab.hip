// fp64 MFMA GEMM lab (not part of the library): C(i,j) = sum_k X[k][i] Y[k][j] on k-major
// operands, lower-triangle (SYRK) or full grids, variants of tile shape / waves / pipeline.
// Build: hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/gemm_lab.hip -o tools/gemm_lab
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <cmath>
#include "../interiorpoint-gpu_amd/csrc/ipm_mfma.h"

typedef double dbl4 __attribute__((ext_vector_type(4)));
#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s at %d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

// BM x BN workgroup tile, WM x WN waves, BK-deep slabs, NSTAGE LDS stages
template <int BM, int BN, int WM, int WN, int BK, bool TRI, int PAD = 0>
__global__ __launch_bounds__(WM * WN * 64) void k_gemm(int n, int K, const double* __restrict__ X, int ldx,
                                                        const double* __restrict__ Y, int ldy,
                                                        double* __restrict__ C, int ldc, int tiles_i, int nblk) {
  constexpr int NT = WM * WN * 64;
  constexpr int TM = BM / WM / 16, TN = BN / WN / 16;   // MFMA tiles per wave
  constexpr int LX = BM + 16, LY = BN + 16;              // padded LDS rows
  constexpr int PX = BK * BM / NT, PY = BK * BN / NT;    // doubles per thread per slab
  static_assert(PX % 2 == 0 && PY % 2 == 0, "pairs");
  __shared__ double sX[2][BK * LX];
  __shared__ double sY[2][BK * LY];
  __shared__ double spad[PAD > 0 ? PAD : 1];
  if (PAD > 0 && threadIdx.x == 0 && n < 0) spad[0] = 0.0;   // keep the pad allocated
  for (int Lp = blockIdx.x; Lp < nblk; Lp += gridDim.x) {
  int bi, bj;
  if (TRI) {
    const int L = Lp;
    int b = (int)((sqrt(8.0 * (double)L + 1.0) - 1.0) * 0.5);
    while ((b + 1) * (b + 2) / 2 <= L) ++b;
    while (b * (b + 1) / 2 > L) --b;
    bi = b; bj = L - b * (b + 1) / 2;   // BM == BN for TRI
  } else {
    bi = Lp % tiles_i; bj = Lp / tiles_i;
  }
  const int I0 = bi * BM, J0 = bj * BN;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int wi = wv % WM, wj = wv / WM;
  dbl4 acc[TN][TM];
#pragma unroll
  for (int a = 0; a < TN; ++a)
#pragma unroll
    for (int b = 0; b < TM; ++b) acc[a][b] = dbl4{0, 0, 0, 0};
  // slab staging: thread covers PX consecutive doubles of one X row (and PY of one Y row)
  constexpr int TPRX = BM / PX, TPRY = BN / PY;
  const int xr = tid / TPRX, xc = (tid % TPRX) * PX;
  const int yr = tid / TPRY, yc = (tid % TPRY) * PY;
  double rx[PX], ry[PY];
  auto gload = [&](int k0) {
    const double2* xp = reinterpret_cast<const double2*>(X + (size_t)(k0 + xr) * ldx + I0 + xc);
    const double2* yp = reinterpret_cast<const double2*>(Y + (size_t)(k0 + yr) * ldy + J0 + yc);
#pragma unroll
    for (int q = 0; q < PX / 2; ++q) { double2 v = xp[q]; rx[2 * q] = v.x; rx[2 * q + 1] = v.y; }
#pragma unroll
    for (int q = 0; q < PY / 2; ++q) { double2 v = yp[q]; ry[2 * q] = v.x; ry[2 * q + 1] = v.y; }
  };
  auto sstore = [&](int buf) {
#pragma unroll
    for (int q = 0; q < PX; ++q) sX[buf][xr * LX + xc + q] = rx[q];
#pragma unroll
    for (int q = 0; q < PY; ++q) sY[buf][yr * LY + yc + q] = ry[q];
  };
  const int nslab = K / BK;
  gload(0); sstore(0);
  if (nslab > 1) gload(BK);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int s = 0; s < nslab; ++s) {
    const int buf = s & 1;
    const double* bx = sX[buf];
    const double* by = sY[buf];
#pragma unroll
    for (int kk = 0; kk < BK / 4; ++kk) {
      double a[TN], b[TM];
#pragma unroll
      for (int t = 0; t < TN; ++t) a[t] = by[(kk * 4 + fk) * LY + wj * (BN / WN) + t * 16 + fr];
#pragma unroll
      for (int t = 0; t < TM; ++t) b[t] = bx[(kk * 4 + fk) * LX + wi * (BM / WM) + t * 16 + fr];
#pragma unroll
      for (int tj = 0; tj < TN; ++tj)
#pragma unroll
        for (int ti = 0; ti < TM; ++ti) acc[tj][ti] = __builtin_amdgcn_mfma_f64_16x16x4f64(a[tj], b[ti], acc[tj][ti], 0, 0, 0);
    }
    if (s + 1 < nslab) {
      sstore(buf ^ 1);
      if (s + 2 < nslab) gload((s + 2) * BK);
    }
    __syncthreads();
  }
#pragma unroll
  for (int tj = 0; tj < TN; ++tj)
#pragma unroll
    for (int ti = 0; ti < TM; ++ti) {
      const int i = I0 + wi * (BM / WM) + ti * 16 + fr;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int j = J0 + wj * (BN / WN) + tj * 16 + fk + 4 * r;
        if (!TRI || i >= j) C[(size_t)j * ldc + i] = acc[tj][ti][r];
      }
    }
  __syncthreads();
  }
}

__global__ void k_ref(int n, int K, const double* X, int ldx, const double* Y, int ldy, double* C, int ldc) {
  int i = blockIdx.x * 256 + threadIdx.x, j = blockIdx.y;
  if (i >= n) return;
  double s = 0;
  for (int k = 0; k < K; ++k) s = fma(X[(size_t)k * ldx + i], Y[(size_t)k * ldy + j], s);
  C[(size_t)j * ldc + i] = s;
}

template <int BM, int BN, int WM, int WN, int BK, bool TRI, int PAD = 0>
void run(const char* name, int n, int K, double* X, double* Y, double* C, double* R, int reps, int grid = 0) {
  const int ti = n / BM, tj = n / BN;
  const int nblk = TRI ? ti * (ti + 1) / 2 : ti * tj;
  auto launch = [&]() {
    hipLaunchKernelGGL((k_gemm<BM, BN, WM, WN, BK, TRI, PAD>), dim3(grid ? grid : nblk), dim3(WM * WN * 64), 0, 0, n, K, X, n, Y, n, C, n, ti, nblk);
  };
  CK(hipMemset(C, 0, (size_t)n * n * 8));
  launch();
  CK(hipDeviceSynchronize());
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  float best = 1e30, tot = 0;
  for (int r = 0; r < reps; ++r) {
    hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
    float ms; hipEventElapsedTime(&ms, a, b); best = std::min(best, ms); tot += ms;
  }
  // check a sample of columns
  std::vector<double> hc((size_t)n * n), hr((size_t)n * n);
  CK(hipMemcpy(hc.data(), C, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), R, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  double err = 0, mx = 0;
  for (int j = 0; j < n; j += 97)
    for (int i = TRI ? j : 0; i < n; ++i) { err = std::max(err, fabs(hc[(size_t)j * n + i] - hr[(size_t)j * n + i])); mx = std::max(mx, fabs(hr[(size_t)j * n + i])); }
  const double fl = TRI ? (double)n * (n + 1) * K : 2.0 * n * n * K;  // tri: useful flops of the triangle
  printf("%-34s n=%d K=%d blocks=%6d  best %.3f ms avg %.3f  %.1f TF/s  relerr %.1e\n", name, n, K, nblk, best,
         tot / reps, fl / best / 1e9, err / mx);
}

void runlib(const char* name, int n, int K, bool tri, bool weight, int remap, double* X, double* C, double* R,
            double* w, int reps, int persist = 0, double beta = 0.0) {
  ipm::GemmArgs a;
  a.ni = n; a.nj = n; a.K = K; a.X = X; a.ldx = n; a.Y = X; a.ldy = n; a.w = weight ? w : nullptr;
  a.C = C; a.ldc = n; a.tri = tri; a.xcd_remap = remap; a.beta = beta; if (beta == 1.0) a.alpha = -1.0;
  CK(hipMemset(C, 0, (size_t)n * n * 8));
  auto L = [&]() { if (persist) ipm::mfma_gemm_launch_persistent(0, a, persist); else ipm::mfma_gemm_launch(0, a); };
  L();
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1; CK(hipEventCreate(&e0)); CK(hipEventCreate(&e1));
  float best = 1e30, tot = 0;
  for (int r = 0; r < reps; ++r) {
    CK(hipEventRecord(e0)); L(); CK(hipEventRecord(e1)); CK(hipEventSynchronize(e1));
    float ms; CK(hipEventElapsedTime(&ms, e0, e1)); best = std::min(best, ms); tot += ms;
  }
  std::vector<double> hc((size_t)n * n), hr((size_t)n * n);
  CK(hipMemcpy(hc.data(), C, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  CK(hipMemcpy(hr.data(), R, (size_t)n * n * 8, hipMemcpyDeviceToHost));
  double err = 0, mx = 0;
  if (!weight && beta == 0.0)
    for (int j = 0; j < n; j += 97)
      for (int i = tri ? j : 0; i < n; ++i) { err = std::max(err, fabs(hc[(size_t)j * n + i] - hr[(size_t)j * n + i])); mx = std::max(mx, fabs(hr[(size_t)j * n + i])); }
  const double fl = tri ? (double)n * (n + 1) * K : 2.0 * n * n * K;
  printf("%-34s n=%d K=%d  best %.3f ms avg %.3f  %.1f TF/s  relerr %.1e\n", name, n, K, best, tot / reps, fl / best / 1e9,
         mx > 0 ? err / mx : 0.0);
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 8192;
  const int K = argc > 2 ? atoi(argv[2]) : 2048;
  double *X, *C, *R;
  CK(hipMalloc(&X, (size_t)K * n * 8)); CK(hipMalloc(&C, (size_t)n * n * 8)); CK(hipMalloc(&R, (size_t)n * n * 8));
  std::vector<double> hx((size_t)K * n);
  srand(1);
  for (auto& v : hx) v = (rand() / (double)RAND_MAX) * 4 - 2;
  CK(hipMemcpy(X, hx.data(), hx.size() * 8, hipMemcpyHostToDevice));
  hipLaunchKernelGGL(k_ref, dim3(n / 256, n), dim3(256), 0, 0, n, K, X, n, X, n, R, n);
  CK(hipDeviceSynchronize());
  const int reps = 5;
  double* w; CK(hipMalloc(&w, (size_t)K * 8));
  { std::vector<double> hw(K, 1.5); CK(hipMemcpy(w, hw.data(), K * 8, hipMemcpyHostToDevice)); }
  runlib("lib tri remap", n, K, true, false, 1, X, C, R, w, reps);
  runlib("lib tri remap beta1", n, K, true, false, 1, X, C, R, w, reps, 0, 1.0);
  runlib("lib persist224 remap", n, K, true, false, 1, X, C, R, w, reps, 224);
  runlib("lib persist224 noremap", n, K, true, false, 0, X, C, R, w, reps, 224);
  runlib("lib persist224 remap beta1", n, K, true, false, 1, X, C, R, w, reps, 224, 1.0);
  runlib("lib persist224 noremap beta1", n, K, true, false, 0, X, C, R, w, reps, 224, 1.0);
  runlib("lib persist256 noremap beta1", n, K, true, false, 0, X, C, R, w, reps, 256, 1.0);
  run<128, 128, 2, 4, 16, true, 2200>("lab w2x4 pad persist224", n, K, X, X, C, R, reps, 224);
  return 0;
}
