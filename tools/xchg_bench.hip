// xchg_bench.hip — diagnostic: floor of the persistent kernel's per-pod exchange on MI355X.
// Every workgroup publishes a tagged 8-byte granule per round and spins until it has seen the
// tag of every workgroup (the persistent kernel's publish → sweep step with no work around
// it).  Reports ns per round for several grid sizes and work amounts between rounds.
//   hipcc -O3 --offload-arch=gfx950 tools/xchg_bench.hip -o /tmp/xchg && /tmp/xchg
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef __attribute__((address_space(1))) uint64_t gu64;

template <int VARIANT>
__device__ __forceinline__ void st(uint64_t* g, uint64_t v) {
  if (VARIANT == 0) __hip_atomic_store((gu64*)g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  else __hip_atomic_store((gu64*)g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <int VARIANT>
__device__ __forceinline__ uint64_t ld(const uint64_t* g) {
  if (VARIANT == 0) return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

// stride: granule spacing in uint64 (16 = 128 B like the kernel)
template <int VARIANT>
__global__ void xchg(uint64_t* gr, int rounds, int stride, int work, uint64_t* out, int* err) {
  const int lane = threadIdx.x & 63;
  const int G = gridDim.x;
  uint64_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  for (int r = 1; r <= rounds; ++r) {
    uint64_t* slot = gr + (int64_t)(r & 1) * 256 * stride;
    const uint64_t tag = (uint64_t)(r & 0xFF);
    if (threadIdx.x < 64) {
      if (lane == 0) st<VARIANT>(slot + (int64_t)blockIdx.x * stride, (tag << 56) | (uint64_t)blockIdx.x);
      const uint64_t ts = __builtin_amdgcn_s_memrealtime();
      for (;;) {
        uint64_t g[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) g[j] = ld<VARIANT>(slot + (int64_t)(lane * 4 + j) * stride);
        bool mine = true;
#pragma unroll
        for (int j = 0; j < 4; ++j) mine &= (lane * 4 + j >= G) || (g[j] >> 56) == tag;
        if (__all(mine)) {
#pragma unroll
          for (int j = 0; j < 4; ++j) acc += g[j] & 0xFFFF;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - ts > 100000000ull) { atomicOr(err, 1); break; }
        __builtin_amdgcn_s_sleep(1);
      }
      // synthetic local work (dependent VALU chain) between rounds
      uint32_t x = (uint32_t)acc;
      for (int k = 0; k < work; ++k) x = x * 1664525u + 1013904223u;
      acc += x & 1;
    }
    __syncthreads();
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  if (threadIdx.x == 0) out[blockIdx.x] = t1 - t0 + (acc & 0);
}

int main() {
  uint64_t *gr, *out;
  int* err;
  const int stride = 16;
  (void)hipMalloc(&gr, 2 * 256 * stride * 8);
  (void)hipMalloc(&out, 256 * 8);
  (void)hipMalloc(&err, 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int rounds = 20000;
  for (int variant = 0; variant < 2; ++variant)
    for (int grid : {2, 8, 32, 64, 128, 256})
      for (int work : {0, 300}) {
        (void)hipMemset(gr, 0, 2 * 256 * stride * 8);
        (void)hipMemset(err, 0, 4);
        (void)hipEventRecord(e0);
        if (variant == 0) hipLaunchKernelGGL(xchg<0>, dim3(grid), dim3(512), 0, 0, gr, rounds, stride, work, out, err);
        else hipLaunchKernelGGL(xchg<1>, dim3(grid), dim3(512), 0, 0, gr, rounds, stride, work, out, err);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        int h_err = 0;
        uint64_t cyc = 0;
        (void)hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost);
        (void)hipMemcpy(&cyc, out, 8, hipMemcpyDeviceToHost);
        printf("scope=%s grid=%3d work=%4d: %8.1f ns/round  %7.0f memtime-cycles/round  err=%d\n",
               variant ? "system" : "agent", grid, work, ms * 1e6 / rounds, (double)cyc / rounds, h_err);
      }
  return 0;
}
