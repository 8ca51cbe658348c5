// Micro-benchmark (diagnostic, not product): cycles per row evaluation of the fast path,
// one 512-thread workgroup per CU, rows in LDS, 8 waves evaluating back-to-back pods.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cmath>

__device__ __forceinline__ int32_t div_floor(double x, double b, double y) {
  double q = trunc(x * y);
  const double r = fma(-q, b, x);
  q = r < 0.0 ? q - 1.0 : (r >= b ? q + 1.0 : q);
  return (int32_t)q;
}
__device__ __forceinline__ double quot(double a, double b, double y) {
  const double q = a * y;
  const double r = fma(-q, b, a);
  return fma(r, y, q);
}

template <int V>
__global__ __launch_bounds__(512) void kb(const double* g, int iters, uint64_t* out, int* sink) {
  __shared__ double ac[512], am[512], zc[512], zm[512], yc[512], ym[512], rc[512], rm[512];
  const int t = threadIdx.x;
  ac[t] = g[t]; am[t] = g[t + 512]; zc[t] = g[t] * 0.25; zm[t] = g[t + 512] * 0.5;
  yc[t] = 1.0 / ac[t]; ym[t] = 1.0 / am[t]; rc[t] = zc[t]; rm[t] = zm[t];
  __syncthreads();
  int32_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int it = 0; it < iters; ++it) {
    const double pc = 100.0 + it, pm = 1000.0 * it;
    const double a_c = ac[t], a_m = am[t], z_c = zc[t], z_m = zm[t], y_c = yc[t], y_m = ym[t];
    const double tc = pc + z_c, tm = pm + z_m;
    int32_t s = 0;
    const bool okc = a_c != 0.0 && tc <= a_c, okm = a_m != 0.0 && tm <= a_m;
    if (V == 0 || V == 1) {
      const int32_t lc = okc ? div_floor((a_c - tc) * 10.0, a_c, y_c) : 0;
      const int32_t lm = okm ? div_floor((a_m - tm) * 10.0, a_m, y_m) : 0;
      s += (lc + lm) / 2;
    }
    if (V == 0 || V == 2) {
      const double fc = a_c != 0.0 ? quot(tc, a_c, y_c) : 1.0;
      const double fm = a_m != 0.0 ? quot(tm, a_m, y_m) : 1.0;
      s += (fc >= 1.0 || fm >= 1.0) ? 0 : (int32_t)((1.0 - fabs(fc - fm)) * 10.0);
    }
    if (V == 3) {  // native divides
      const double fc = tc / a_c, fm = tm / a_m;
      s += (fc >= 1.0 || fm >= 1.0) ? 0 : (int32_t)((1.0 - fabs(fc - fm)) * 10.0);
      s += (int32_t)((a_c - tc) * 10.0 / a_c);
    }
    acc += s;
    if (V == 4) acc += (tc <= a_c) + (tm <= a_m);
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (acc == 0x7fffffff) sink[t] = acc;
  if (t % 64 == 0) out[blockIdx.x * 8 + t / 64] = t1 - t0;
}

int main() {
  const int B = 256, iters = 2000;
  double h[1024];
  for (int i = 0; i < 1024; ++i) h[i] = (i < 512) ? 16000.0 + 1000 * (i % 7) : 68719476736.0 * (1 + i % 3);
  double* g; uint64_t* o; int* s;
  hipMalloc(&g, sizeof h); hipMalloc(&o, B * 8 * 8); hipMalloc(&s, 4 * 512);
  hipMemcpy(g, h, sizeof h, hipMemcpyHostToDevice);
  const char* names[] = {"LR+BRA", "LR", "BRA", "native-div", "compare-only"};
  for (int bs : {512, 64})
  for (int v = 0; v < 5; ++v) {
    for (int rep = 0; rep < 2; ++rep) {
      switch (v) {
        case 0: hipLaunchKernelGGL(kb<0>, dim3(B), dim3(bs), 0, 0, g, iters, o, s); break;
        case 1: hipLaunchKernelGGL(kb<1>, dim3(B), dim3(bs), 0, 0, g, iters, o, s); break;
        case 2: hipLaunchKernelGGL(kb<2>, dim3(B), dim3(bs), 0, 0, g, iters, o, s); break;
        case 3: hipLaunchKernelGGL(kb<3>, dim3(B), dim3(bs), 0, 0, g, iters, o, s); break;
        case 4: hipLaunchKernelGGL(kb<4>, dim3(B), dim3(bs), 0, 0, g, iters, o, s); break;
      }
      hipDeviceSynchronize();
    }
    uint64_t ho[B * 8];
    hipMemcpy(ho, o, sizeof ho, hipMemcpyDeviceToHost);
    const int nw = bs / 64;
    double m = 0; for (int b = 0; b < B; ++b) for (int w = 0; w < nw; ++w) m += ho[b * 8 + w];
    printf("%-14s %.1f cycles per iteration (%d waves/CU)\n", names[v], m / (B * nw) / iters, nw);
  }
  return 0;
}
