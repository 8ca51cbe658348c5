// xchg_bench2.hip — diagnostic: the cross-CU hand-off floors behind the C3 persistent kernel's
// per-pod cycle, for the protocol decision of DESIGN.md §4 ("Where the C3 time goes").
//   mode 0 "bcast": the current protocol's critical hop.  Every workgroup has published its
//     granule of round r early (tag r); one rotating "owner" (a data-dependent workgroup) publishes
//     the late fix granule of round r only once it has seen round r-1 complete; every workgroup
//     sweeps all granules + the fix (NREP replicas, like ksim_pfast_kernel) and then publishes its
//     granule of round r+1.  ns/round = one-to-all publish -> observe + sweep.
//   mode 1 "baton": one-to-one hand-off.  The holder of round r waits for its mailbox tag r and
//     for every workgroup's granule of round r (published ahead, bounded by a progress word the
//     holders advance), then passes the baton to the next data-dependent holder's mailbox.
//     ns/round = mailbox hop + the holder's (already in flight) sweep.
//   hipcc -O3 --offload-arch=gfx950 tools/xchg_bench2.hip -o /tmp/xchg2 && /tmp/xchg2
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef __attribute__((address_space(1))) uint64_t gu64;

__device__ __forceinline__ void st(uint64_t* g, uint64_t v) {
  __hip_atomic_store((gu64*)g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t ld(const uint64_t* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

constexpr int MAXB = 4, MAXG = 256, NSLOT = 4, NREP = 8, REP = 2112;
constexpr uint64_t LIMIT = 100000000ull;  // 1 s of s_memrealtime

__device__ __forceinline__ int owner_of(int r, int G) { return (int)(((uint32_t)r * 2654435761u) >> 8) % G; }

// mode 0: [rep][slot][pos] granules + [rep][slot] fix at the end of each replica
__global__ __launch_bounds__(512) void bcast(uint64_t* gr, int rounds, int* err, uint64_t* out) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x, G = gridDim.x, me = blockIdx.x;
  uint64_t* my = gr + (me % NREP) * REP;
  auto gpos = [&](int slot, int b) { return slot * MAXG + (b % MAXB) * 64 + b / MAXB; };
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  // round 1's granule
  if (lane < NREP) st(gr + lane * REP + gpos(1 % NSLOT, me), (1ull << 56) | me);
  uint64_t acc = 0;
  for (int r = 1; r <= rounds; ++r) {
    const int slot = r % NSLOT, own = owner_of(r, G);
    const uint64_t tag = (uint64_t)(r & 0xFF);
    if (me == own && lane < NREP) st(gr + lane * REP + NSLOT * MAXG + slot * 16, (tag << 56) | 7);
    const uint64_t ts = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      uint64_t g[MAXB];
#pragma unroll
      for (int j = 0; j < MAXB; ++j) g[j] = ld(my + slot * MAXG + j * 64 + lane);
      const uint64_t fx = ld(my + NSLOT * MAXG + slot * 16);
      bool ok = (fx >> 56) == tag;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) ok &= (lane * MAXB + j >= G) || (g[j] >> 56) == tag;
      if (__all(ok)) {
#pragma unroll
        for (int j = 0; j < MAXB; ++j) acc += g[j] & 0xFF;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - ts > LIMIT) { atomicOr(err, 1); return; }
      __builtin_amdgcn_s_sleep(1);
    }
    // granule of round r + 1 (spec: published a round ahead, like the row waves' publish)
    if (lane < NREP) st(gr + lane * REP + gpos((r + 1) % NSLOT, me), ((uint64_t)((r + 1) & 0xFF) << 56) | me);
  }
  if (lane == 0) out[me] = __builtin_amdgcn_s_memtime() - t0 + (acc & 0);
}

// mode 2/3: mode 0 with pipelined polling — DEPTH sweeps in flight, the oldest checked while the
// younger ones travel, so a granule that lands is seen about one round trip / DEPTH later.
template <int DEPTH>
__global__ __launch_bounds__(512) void bcast_pipe(uint64_t* gr, int rounds, int* err, uint64_t* out) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x, G = gridDim.x, me = blockIdx.x;
  uint64_t* my = gr + (me % NREP) * REP;
  auto gpos = [&](int slot, int b) { return slot * MAXG + (b % MAXB) * 64 + b / MAXB; };
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (lane < NREP) st(gr + lane * REP + gpos(1 % NSLOT, me), (1ull << 56) | me);
  uint64_t acc = 0;
  for (int r = 1; r <= rounds; ++r) {
    const int slot = r % NSLOT, own = owner_of(r, G);
    const uint64_t tag = (uint64_t)(r & 0xFF);
    if (me == own && lane < NREP) st(gr + lane * REP + NSLOT * MAXG + slot * 16, (tag << 56) | 7);
    const uint64_t ts = __builtin_amdgcn_s_memrealtime();
    uint64_t g[DEPTH][MAXB + 1];
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
#pragma unroll
      for (int j = 0; j < MAXB; ++j) g[d][j] = ld(my + slot * MAXG + j * 64 + lane);
      g[d][MAXB] = ld(my + NSLOT * MAXG + slot * 16);
      if (d + 1 < DEPTH) __builtin_amdgcn_s_sleep(2);
    }
    for (;;) {
      bool ok = (g[0][MAXB] >> 56) == tag;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) ok &= (lane * MAXB + j >= G) || (g[0][j] >> 56) == tag;
      if (__all(ok)) {
#pragma unroll
        for (int j = 0; j < MAXB; ++j) acc += g[0][j] & 0xFF;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - ts > LIMIT) { atomicOr(err, 1); return; }
#pragma unroll
      for (int d = 0; d + 1 < DEPTH; ++d)
#pragma unroll
        for (int j = 0; j <= MAXB; ++j) g[d][j] = g[d + 1][j];
#pragma unroll
      for (int j = 0; j < MAXB; ++j) g[DEPTH - 1][j] = ld(my + slot * MAXG + j * 64 + lane);
      g[DEPTH - 1][MAXB] = ld(my + NSLOT * MAXG + slot * 16);
    }
    if (lane < NREP) st(gr + lane * REP + gpos((r + 1) % NSLOT, me), ((uint64_t)((r + 1) & 0xFF) << 56) | me);
  }
  if (lane == 0) out[me] = __builtin_amdgcn_s_memtime() - t0 + (acc & 0);
}

// mode 5/6: the split sweep of the reworked ksim_pfast control wave — every granule but the
// previous owner's (published a round ahead) is swept first, then only the late fix granule is
// polled, by one 8-byte load per iteration (mode 6: no s_sleep between polls).
template <bool NOSLEEP>
__global__ __launch_bounds__(512) void bcast_split(uint64_t* gr, int rounds, int* err, uint64_t* out) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x, G = gridDim.x, me = blockIdx.x;
  uint64_t* my = gr + (me % NREP) * REP;
  auto gpos = [&](int slot, int b) { return slot * MAXG + (b % MAXB) * 64 + b / MAXB; };
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (lane < NREP) st(gr + lane * REP + gpos(1 % NSLOT, me), (1ull << 56) | me);
  uint64_t acc = 0;
  for (int r = 1; r <= rounds; ++r) {
    const int slot = r % NSLOT, own = owner_of(r, G);
    const uint64_t tag = (uint64_t)(r & 0xFF);
    if (me == own && lane < NREP) st(gr + lane * REP + NSLOT * MAXG + slot * 16, (tag << 56) | 7);
    const uint64_t ts = __builtin_amdgcn_s_memrealtime();
    for (;;) {
      uint64_t g[MAXB];
#pragma unroll
      for (int j = 0; j < MAXB; ++j) g[j] = ld(my + slot * MAXG + j * 64 + lane);
      bool ok = true;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) ok &= (lane * MAXB + j >= G) || (g[j] >> 56) == tag;
      if (__all(ok)) {
#pragma unroll
        for (int j = 0; j < MAXB; ++j) acc += g[j] & 0xFF;
        break;
      }
      if (__builtin_amdgcn_s_memrealtime() - ts > LIMIT) { atomicOr(err, 1); return; }
      __builtin_amdgcn_s_sleep(1);
    }
    for (;;) {
      const uint32_t fx = (uint32_t)__builtin_amdgcn_readfirstlane((int)(ld(my + NSLOT * MAXG + slot * 16) >> 32));
      if ((uint64_t)(fx >> 24) == tag) break;
      if (__builtin_amdgcn_s_memrealtime() - ts > LIMIT) { atomicOr(err, 1); return; }
      if (!NOSLEEP) __builtin_amdgcn_s_sleep(1);
    }
    if (lane < NREP) st(gr + lane * REP + gpos((r + 1) % NSLOT, me), ((uint64_t)((r + 1) & 0xFF) << 56) | me);
  }
  if (lane == 0) out[me] = __builtin_amdgcn_s_memtime() - t0 + (acc & 0);
}

// mode 1: granules [slot][pos] (one copy, NREP replicas), mailboxes [G] 128 B apart, progress word
__global__ __launch_bounds__(512) void baton(uint64_t* gr, uint64_t* mbox, uint64_t* prog, int rounds, int* err,
                                             uint64_t* out) {
  if (threadIdx.x >= 64) return;
  const int lane = threadIdx.x, G = gridDim.x, me = blockIdx.x;
  uint64_t* my = gr + (me % NREP) * REP;
  auto gpos = [&](int slot, int b) { return slot * MAXG + (b % MAXB) * 64 + b / MAXB; };
  int pub = 1;         // next round this workgroup publishes a granule for
  int64_t done = 0;    // last completed round it knows of
  uint64_t acc = 0;
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  if (me == owner_of(1, G) && lane == 0) st(mbox + me * 16, 1);
  const uint64_t ts0 = __builtin_amdgcn_s_memrealtime();
  int r = 1;  // round this workgroup waits for as a holder (any round it may hold)
  while (done < rounds) {
    // publish ahead: rounds up to done + NSLOT - 1
    while (pub <= rounds && pub < done + NSLOT) {
      if (lane < NREP) st(gr + lane * REP + gpos(pub % NSLOT, me), ((uint64_t)(pub & 0xFF) << 56) | me);
      ++pub;
    }
    const uint64_t m = ld(mbox + me * 16);
    const int64_t pg = (int64_t)ld(prog);
    done = pg > done ? pg : done;
    // the baton of round m is sent only once round m - 1 is complete (the progress word may lag)
    r = (int64_t)m > done ? (int)m : (int)done + 1;
    if ((int64_t)m == r && r <= rounds) {
      // holder of round r: every granule of round r, then pass the baton
      const int slot = r % NSLOT;
      const uint64_t tag = (uint64_t)(r & 0xFF);
      for (;;) {
        uint64_t g[MAXB];
#pragma unroll
        for (int j = 0; j < MAXB; ++j) g[j] = ld(my + slot * MAXG + j * 64 + lane);
        bool ok = true;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) ok &= (lane * MAXB + j >= G) || (g[j] >> 56) == tag;
        if (__all(ok)) {
#pragma unroll
          for (int j = 0; j < MAXB; ++j) acc += g[j] & 0xFF;
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - ts0 > 10 * LIMIT) { atomicOr(err, 2); return; }
      }
      if (lane == 0) {
        if (r < rounds) st(mbox + owner_of(r + 1, G) * 16, (uint64_t)(r + 1));
        st(prog, (uint64_t)r);
      }
      done = r;
      continue;
    }
    if (__builtin_amdgcn_s_memrealtime() - ts0 > 10 * LIMIT) { atomicOr(err, 4); return; }
    __builtin_amdgcn_s_sleep(1);
  }
  if (lane == 0) out[me] = __builtin_amdgcn_s_memtime() - t0 + (acc & 0);
}

int main() {
  uint64_t *gr, *mbox, *prog, *out;
  int* err;
  const size_t gbytes = (size_t)NREP * REP * 8;
  (void)hipMalloc(&gr, gbytes);
  (void)hipMalloc(&mbox, 256 * 16 * 8);
  (void)hipMalloc(&prog, 64);
  (void)hipMalloc(&out, 256 * 8);
  (void)hipMalloc(&err, 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int rounds = 20000;
  for (int mode = 0; mode < 7; ++mode)
    for (int grid : {8, 64, 128, 256}) {
      (void)hipMemset(gr, 0, gbytes);
      (void)hipMemset(mbox, 0, 256 * 16 * 8);
      (void)hipMemset(prog, 0, 64);
      (void)hipMemset(err, 0, 4);
      (void)hipEventRecord(e0);
      if (mode == 0) hipLaunchKernelGGL(bcast, dim3(grid), dim3(512), 0, 0, gr, rounds, err, out);
      else if (mode == 1) hipLaunchKernelGGL(baton, dim3(grid), dim3(512), 0, 0, gr, mbox, prog, rounds, err, out);
      else if (mode == 2) hipLaunchKernelGGL(bcast_pipe<2>, dim3(grid), dim3(512), 0, 0, gr, rounds, err, out);
      else if (mode == 3) hipLaunchKernelGGL(bcast_pipe<3>, dim3(grid), dim3(512), 0, 0, gr, rounds, err, out);
      else if (mode == 4) hipLaunchKernelGGL(bcast_pipe<4>, dim3(grid), dim3(512), 0, 0, gr, rounds, err, out);
      else if (mode == 5) hipLaunchKernelGGL(bcast_split<false>, dim3(grid), dim3(512), 0, 0, gr, rounds, err, out);
      else hipLaunchKernelGGL(bcast_split<true>, dim3(grid), dim3(512), 0, 0, gr, rounds, err, out);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms = 0;
      (void)hipEventElapsedTime(&ms, e0, e1);
      int h_err = 0;
      (void)hipMemcpy(&h_err, err, 4, hipMemcpyDeviceToHost);
      static const char* names[7] = {"bcast", "baton", "bcast-pipe2", "bcast-pipe3", "bcast-pipe4", "bcast-split",
                                      "bcast-split-nosleep"};
      printf("mode=%s grid=%3d: %8.1f ns/round  err=%d\n", names[mode], grid, ms * 1e6 / rounds, h_err);
      fflush(stdout);
      if (h_err) return 1;
    }
  return 0;
}
