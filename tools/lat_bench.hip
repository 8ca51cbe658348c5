// Micro-benchmark (diagnostic): dependent-chain latency of single ops on gfx950, one wave.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
template <int V>
__global__ void kl(double* d, float* f, int* ii, int n, uint64_t* out) {
  double x = d[threadIdx.x], y = d[threadIdx.x + 64];
  float a = f[threadIdx.x], b = f[threadIdx.x + 64];
  int p = ii[threadIdx.x], q = ii[threadIdx.x + 64];
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int i = 0; i < n; ++i) {
#pragma unroll
    for (int u = 0; u < 16; ++u) {
    if (V == 0) x = fma(x, y, 0.5);
    if (V == 1) a = fmaf(a, b, 0.5f);
    if (V == 2) p = p * q + 1;
    if (V == 3) x = x * y;
    if (V == 4) { x = trunc(x * y); }
    if (V == 5) { x = x * y + (double)i; }
    if (V == 6) { a = a * b; }
    if (V == 7) { p = p ^ (p << 1); }
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  d[threadIdx.x] = x; f[threadIdx.x] = a; ii[threadIdx.x] = p;
  if (threadIdx.x == 0) out[V] = t1 - t0;
}
int main() {
  double* d; float* f; int* ii; uint64_t* o;
  hipMalloc(&d, 1024); hipMalloc(&f, 1024); hipMalloc(&ii, 1024); hipMalloc(&o, 64);
  hipMemset(d, 0, 1024); hipMemset(f, 0, 1024); hipMemset(ii, 0, 1024);
  const int n = 10000;
  for (int rep = 0; rep < 2; ++rep) {
    hipLaunchKernelGGL(kl<0>, 1, 64, 0, 0, d, f, ii, n, o);
    hipLaunchKernelGGL(kl<1>, 1, 64, 0, 0, d, f, ii, n, o);
    hipLaunchKernelGGL(kl<2>, 1, 64, 0, 0, d, f, ii, n, o);
    hipLaunchKernelGGL(kl<3>, 1, 64, 0, 0, d, f, ii, n, o);
    hipLaunchKernelGGL(kl<4>, 1, 64, 0, 0, d, f, ii, n, o);
    hipLaunchKernelGGL(kl<5>, 1, 64, 0, 0, d, f, ii, n, o);
    hipLaunchKernelGGL(kl<6>, 1, 64, 0, 0, d, f, ii, n, o);
    hipLaunchKernelGGL(kl<7>, 1, 64, 0, 0, d, f, ii, n, o);
    hipDeviceSynchronize();
  }
  uint64_t h[8];
  hipMemcpy(h, o, 64, hipMemcpyDeviceToHost);
  const char* nm[] = {"fma_f64", "fma_f32", "mul_lo_i32+add", "mul_f64", "mul_f64+trunc", "mul_f64+add_f64(cvt)", "mul_f32", "xor+shl i32"};
  for (int v = 0; v < 8; ++v) printf("%-26s %.2f cycles per dependent step\n", nm[v], (double)h[v] / n / 16);
  return 0;
}
