// ksim_pfast.hip — persistent-kernel mode specialised for resource-only pods (the C1/C3/C4/C5
// pod shape, ksim_is_fast_pod): used for a ksim_schedule() call whenever every pod of the call
// qualifies and every cpu / memory quantity of the nodes and pods is below 2^48 (host check);
// ksim_persistent.hip handles everything else.  A commit that takes a node's quantity to 2^48
// or beyond stops the kernel before the next pod (uniformly, through the correction granule)
// and the host finishes the call with the general kernel.
//
// Same protocol as ksim_persistent.hip — workgroup b keeps the name-rank range
// [b*chunk, (b+1)*chunk) in LDS, one control wave (wave 0) decides every pod redundantly from
// the tagged 8-byte granules all workgroups publish, seven row waves evaluate pod p+1 while
// the control wave decides pod p — with a shorter critical path:
//
//  * float64 rows.  Every quantity is an integer below 2^48 and every sum below 2^49, so sums, compares
//    and the products below are exact in float64 and the Go int64 arithmetic is reproduced
//    without 64-bit integer emulation.  Each row keeps y = RN(1/alloc) (alloc is static):
//    LeastRequested / MostRequested floor(10x / cap) = trunc(x*y) corrected by the exact
//    remainder fma(-q, cap, x) (least_requested.go:44-53, most_requested.go:45-55);
//    BalancedResourceAllocation's float64(req)/float64(cap) (balanced_resource_allocation.go:
//    39-61) = Markstein's RN(a/b): q = a*y, r = fma(-q, b, a) (exact), RN(q + r*y) — the
//    correctly rounded quotient, bit-identical to the IEEE divide Go performs (y within half an
//    ulp of 1/b, q within one ulp of a/b, no over/underflow).
//  * the row waves also evaluate pod p+1 against "row + pod p" for every row (two independent
//    evaluations per lane, overlapped), so the owner of pod p's node finds the post-commit
//    evaluation in LDS;
//  * O(1) owner fix-up: the row waves keep the workgroup's top two (score, count) pairs of
//    pod p+1, so the owner removes the committed row's pre-commit evaluation and adds its
//    post-commit one with scalar arithmetic, publishes, and only then commits the row;
//  * one prefix scan per decision: counts at the maximum give C (= its total) and the
//    workgroup holding the ix-th match from the top (core/generic_scheduler.go:183-198).
#include <algorithm>

#include "ksim_f64.h"
#include "ksim_fast.h"
#include "ksim_tree.h"
#include "ksim_wave.h"

using namespace kf64;

namespace {

#ifndef KSIM_PF_BS
#define KSIM_PF_BS 512  // threads per workgroup (diagnostic variants: 256 = control + 3 row waves)
#endif
constexpr int BS = KSIM_PF_BS;
constexpr int NW = BS / 64;     // waves per workgroup
constexpr int RW = NW - 1;      // row waves
constexpr int RT = RW * 64;     // row threads
constexpr int MAXB = 4;         // workgroups per sweep lane (grid <= 256)
constexpr int MAXG = 64 * MAXB;
constexpr int NSLOT = 4;        // granule slots (pod mod NSLOT)
constexpr int FIXSTRIDE = 16;   // fix granules 128 B apart
constexpr int RING = 16;        // pod-descriptor ring slots in LDS
constexpr int RING_FILL = 8;    // descriptors fetched per refill
constexpr uint64_t SPIN_LIMIT_TICKS = 200000000ull;  // s_memrealtime at 100 MHz = 2 s
constexpr int ANSLOT = 8;       // aggregate slots per rank (pod mod ANSLOT)

typedef __attribute__((address_space(1))) uint64_t gu64;

// cross-device exchange (fine-grained memory written by peers over xGMI)
__device__ __forceinline__ void sys_store(uint64_t* g, uint64_t v) {
  __hip_atomic_store(g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t sys_load(const uint64_t* g) {
  return __hip_atomic_load(g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}

__device__ __forceinline__ void store_granule(uint64_t* g, uint64_t v) {
  __hip_atomic_store((gu64*)g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_granule(const uint64_t* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// [slot][pos(b)], pos(b) = (b % MAXB) * 64 + b / MAXB: the sweep's j-th load of lane l is
// workgroup l*MAXB + j and each load instruction is 512 contiguous bytes.
__device__ __forceinline__ uint64_t* spec_at(uint64_t* gr, int slot, int b) {
  return gr + slot * MAXG + (b % MAXB) * 64 + b / MAXB;
}
__device__ __forceinline__ uint64_t* fix_at(uint64_t* gr, int slot) { return gr + NSLOT * MAXG + slot * FIXSTRIDE; }
// Every granule is written to NREP replicas of the whole array (lane r of the publishing wave
// writes replica r) and workgroup b polls replica b % NREP: the 256 pollers spread over NREP
// sets of lines instead of all sweeping the same 2 KB.
#ifndef KSIM_NREP
#define KSIM_NREP 8
#endif
constexpr int NREP = KSIM_NREP;

constexpr int REP_STRIDE = 2112;  // uint64 words between replicas (16.5 KB, > one replica)
static_assert(NSLOT * MAXG + NSLOT * FIXSTRIDE <= REP_STRIDE, "replica overlap");

// granule: tag:8 | stop:1 | fit:13 | count:13 | score:29 (two's complement, -1 = no fit node;
// scores < 2^27, host-checked); stop (correction granules only): the committed node left the
// exact float64 range, end the call before this pod.  A workgroup owns < 8192 rows.
constexpr double EXACT_LIM = 281474976710656.0;  // 2^48
__device__ __forceinline__ uint32_t gtag(uint64_t v) { return (uint32_t)(v >> 56); }
__device__ __forceinline__ bool gstop(uint64_t v) { return (v >> 55) & 1; }
__device__ __forceinline__ int32_t gfit(uint64_t v) { return (int32_t)((v >> 42) & 0x1FFF); }
__device__ __forceinline__ int32_t gcnt(uint64_t v) { return (int32_t)((v >> 29) & 0x1FFF); }
__device__ __forceinline__ int32_t gscore(uint64_t v) { return ((int32_t)((uint32_t)v << 3)) >> 3; }
__device__ __forceinline__ uint64_t gpack(uint64_t tag, int32_t f, int32_t n, int32_t m) {
  return (tag << 56) | ((uint64_t)(uint32_t)f << 42) | ((uint64_t)(uint32_t)n << 29) | ((uint64_t)(uint32_t)m & 0x1FFFFFFFull);
}

// Workgroup barrier ordering LDS only: __syncthreads' fence would also drain this wave's
// outstanding global operations (the granule store just published, a descriptor prefetch),
// which other waves of the workgroup never read.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// critical-path probes (diagnostic builds only, tools/build_variants): ~500-cycle delay at point k
#ifdef KSIM_PROBE
#define PROBE(k) do { if (KSIM_PROBE == (k)) __builtin_amdgcn_s_sleep(8); } while (0)
#else
#define PROBE(k) do { } while (0)
#endif

#ifdef KSIM_STAMPS
#define STAMP(k)                                       \
  do {                                                 \
    const uint64_t t_ = __builtin_amdgcn_s_memtime(); \
    st_acc[k] += t_ - t_prev;                         \
    t_prev = t_;                                      \
  } while (0)
#define OSTAMP(k)                                                          \
  do {                                                                     \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                     \
    if (lane == 0) atomicAdd((unsigned long long*)&a.dbg[k], t_ - o_prev); \
    o_prev = t_;                                                           \
  } while (0)
#else
#define STAMP(k) \
  do {           \
  } while (0)
#define OSTAMP(k) \
  do {            \
  } while (0)
#endif

}  // namespace

// Kernel arguments: only what the fast path touches.
struct PfArgs {
  int64_t n, chunk, first, end;
  const int64_t* alloc_cpu;
  const int64_t* alloc_mem;
  const int32_t* allowed_pods;
  const uint32_t* flags;
  int64_t* req_cpu;
  int64_t* req_mem;
  int64_t* nz_cpu;
  int64_t* nz_mem;
  int32_t* pod_count;
  const ksim_pod* pods;
  uint64_t* counter;
  int64_t* cursor;
  int32_t* out_node;
  int32_t* out_reasons;
  int32_t* err;
  uint64_t* dbg;
  uint64_t* granules;
  uint32_t preds;
  int32_t no_prio, collect;
  int32_t wl, wm, wb;  // map weights (host-checked: sum x 10 < 2^27)
  // node-sharded mode (world > 1): this rank holds global name ranks
  // [node_base, node_base + n); per pod, workgroup 0 publishes the rank's aggregate to every
  // rank's exchange buffer (over xGMI) and every workgroup combines the world's aggregates
  int32_t rank, world;
  int64_t node_base;
  uint32_t xtag_base;                 // exchange tag of pod first - 1 (host: running pod count)
  uint64_t* xchg;                     // this rank's aggregate slots [ANSLOT][KSIM_MAX_RANKS][4]
  uint64_t* peers[KSIM_MAX_RANKS];    // every rank's exchange buffer as mapped here (self included)
  uint64_t start_ticks;               // bound of the first pod's cross-rank wait (KsimShard)
  // streaming form (tables beyond the LDS budget): float64 image of the table in HBM,
  // [6][n] = alloc cpu, alloc mem, requested cpu, mem, non-zero cpu, mem
  double* mirror;
  // cached form (LDS rows, map-only policies, ncls > 0): every (tree class, row) evaluation is
  // kept in LDS and only the committed row is re-evaluated — see "Cached form" below
  const int32_t* tcls;            // [pods] tree class of each queued pod (resource-only key)
  const KsimTreeClass* tclass;    // [ncls] the class's predicate / priority inputs
  int32_t ncls;
};

namespace {

struct FRows {  // LDS image of the owned rows (SoA)
  double *ac, *am, *rc, *rm, *zc, *zm, *yc, *ym;
  int32_t *allowed, *count;
  uint32_t* fl;
  int32_t* ev;    // [2][chunk]: evaluation of pod p (parity p & 1), -1 = does not fit
  int32_t* ev2;   // [chunk]: evaluation of pod p+1 against row + pod p
  uint32_t* rm2;  // [chunk]: ... its reason mask
  uint32_t* rma;  // STREAM: [2][chunk] reason mask of ev (registers in the LDS form)
  int16_t* cache; // CACHE: [ncls][chunk] evaluation of tree class k on row j as it stands
};

constexpr int LDS_ROW_BYTES = 8 * 8 + 8 * 4;  // 96: 8 float64 + allowed, count, flags, ev[2], ev2, rm2, top_list
constexpr int LDS_ROW_BYTES_STREAM = 7 * 4;   // ev[2], ev2, rm2, top_list, rma[2] (rows stream from HBM)

extern __shared__ __attribute__((aligned(16))) char kf_smem[];

// STREAM: the rows are the workgroup's slice of the HBM float64 image (+ the int32 columns
// themselves); only the per-row evaluations live in LDS.
template <bool STREAM>
__device__ __forceinline__ FRows carve(int rows, const PfArgs& a, int64_t lo) {
  FRows r;
  if (STREAM) {
    double* m = a.mirror + lo;
    const int64_t n = a.n;
    r.ac = m; r.am = m + n; r.rc = m + 2 * n; r.rm = m + 3 * n;
    r.zc = m + 4 * n; r.zm = m + 5 * n; r.yc = nullptr; r.ym = nullptr;
    r.allowed = const_cast<int32_t*>(a.allowed_pods) + lo;
    r.count = a.pod_count + lo;
    r.fl = const_cast<uint32_t*>(a.flags) + lo;
    int32_t* q = reinterpret_cast<int32_t*>(kf_smem);
    r.ev = q;
    r.ev2 = q + 2 * rows;
    r.rm2 = reinterpret_cast<uint32_t*>(q + 3 * rows);
    r.rma = r.rm2 + 2 * rows;  // after top_list
    r.cache = nullptr;
    return r;
  }
  double* d = reinterpret_cast<double*>(kf_smem);
  r.ac = d; r.am = d + rows; r.rc = d + 2 * rows; r.rm = d + 3 * rows;
  r.zc = d + 4 * rows; r.zm = d + 5 * rows; r.yc = d + 6 * rows; r.ym = d + 7 * rows;
  int32_t* q = reinterpret_cast<int32_t*>(d + 8 * rows);
  r.allowed = q; r.count = q + rows;
  r.fl = reinterpret_cast<uint32_t*>(q + 2 * rows);
  r.ev = q + 3 * rows;
  r.ev2 = q + 5 * rows;
  r.rm2 = reinterpret_cast<uint32_t*>(q + 6 * rows);
  r.cache = reinterpret_cast<int16_t*>(q + 8 * rows);  // after top_list (q + 7 rows)
  return r;
}

// STREAM, control wave: row j read from L2 (agent-scope relaxed loads, past this CU's L1), so a
// store another wave of the workgroup completed before the last barrier is seen
typedef __attribute__((address_space(1))) const uint64_t cgu64;
typedef __attribute__((address_space(1))) const int32_t cgi32;
__device__ __forceinline__ double ld_l2(const double* p) {
  return __builtin_bit_cast(double, __hip_atomic_load((cgu64*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}
__device__ __forceinline__ int32_t ld_l2(const int32_t* p) {
  return __hip_atomic_load((cgi32*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ FRow load_frow_l2(const FRows& R, int32_t j) {
  FRow r;
  r.ac = ld_l2(R.ac + j); r.am = ld_l2(R.am + j); r.rc = ld_l2(R.rc + j); r.rm = ld_l2(R.rm + j);
  r.zc = ld_l2(R.zc + j); r.zm = ld_l2(R.zm + j);
  r.yc = r.ac != 0.0 ? 1.0 / r.ac : 0.0;
  r.ym = r.am != 0.0 ? 1.0 / r.am : 0.0;
  r.allowed = ld_l2(R.allowed + j); r.count = ld_l2(R.count + j);
  r.fl = (uint32_t)ld_l2(reinterpret_cast<const int32_t*>(R.fl) + j);
  return r;
}

// STREAM: y = RN(1/alloc) is recomputed (IEEE divide) instead of read, so a row costs exactly
// the 60 algorithmic bytes: 6 x 8 (alloc, requested, non-zero requested cpu / mem) + 3 x 4.
template <bool STREAM>
__device__ __forceinline__ FRow load_frow(const FRows& R, int32_t j) {
  FRow r;
  r.ac = R.ac[j]; r.am = R.am[j]; r.rc = R.rc[j]; r.rm = R.rm[j]; r.zc = R.zc[j]; r.zm = R.zm[j];
  if (STREAM) {
    r.yc = r.ac != 0.0 ? 1.0 / r.ac : 0.0;
    r.ym = r.am != 0.0 ? 1.0 / r.am : 0.0;
  } else {
    r.yc = R.yc[j]; r.ym = R.ym[j];
  }
  r.allowed = R.allowed[j]; r.count = R.count[j]; r.fl = R.fl[j];
  return r;
}

// top-two (score, count) statistics of a set of evaluations
struct Top2 {
  int32_t f, m1, c1, m2, c2;
};

}  // namespace

template <int NPT, bool STREAM, bool CACHE>
__global__ __launch_bounds__(BS) void ksim_pfast_kernel(PfArgs a) {
  static_assert(!(STREAM && CACHE), "the cached form keeps the rows in LDS");
  __shared__ int32_t s_wst[2][RW][5];         // per row wave: fit, m1, c1, m2, c2 (by pod parity)
  __shared__ uint64_t s_bm[2][NPT][RW];       // per 64-row segment: rows at the wave maximum
  __shared__ int32_t s_wg[2][5];              // workgroup top-two of the pod
  __shared__ int32_t s_fix[2][2];             // {row the owner corrected (-1 none), its reason mask}
  __shared__ int32_t s_hist[KSIM_NREASONS];
  __shared__ int32_t s_mode[2], s_own[2];     // by pod parity: read after the barrier, rewritten two pods later
  __shared__ int32_t s_arr;
  // STREAM: commit of pod p deferred to the row waves of the next iteration (by pod parity):
  // row (-1 none) and the AddPod deltas (add cpu, add mem, non-zero cpu, non-zero mem)
  __shared__ int32_t s_prow[2];
  __shared__ double s_pdel[2][4];
  __shared__ double s_pval[4];   // STREAM: the deferred-commit row's dynamic values after applying it
  __shared__ int32_t s_pcnt;
  __shared__ __attribute__((aligned(16))) ksim_pod s_pod[RING];
  __shared__ int32_t s_pcls[CACHE ? RING : 1];                              // CACHE: tree class of each ring slot
  __shared__ KsimTreeClass s_tcl[CACHE ? KSIM_TREE_MAX_CLASSES : 1];       // CACHE: the class inputs
#ifdef KSIM_STAMPS
  uint64_t st_acc[16] = {};
#endif

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int rt = tid - 64;
  const int G = gridDim.x;
  const int me = blockIdx.x;
  const int64_t chunk = a.chunk;
  const int64_t lo = (int64_t)me * chunk;
  const int64_t hi = (lo + chunk < a.n) ? lo + chunk : a.n;
  const int32_t nrows = (int32_t)(hi - lo);
  const FRows R = carve<STREAM>((int)chunk, a, lo);
  const uint32_t preds = a.preds;
  const bool no_prio = a.no_prio != 0;
  const EvCfg EC = make_evcfg(preds, no_prio, a.wl, a.wm, a.wb);
  int32_t* const top_list = reinterpret_cast<int32_t*>(R.rm2 + chunk);  // STREAM: [chunk] rows at the workgroup maximum, from the top
  uint64_t* const granules = a.granules;
  constexpr int NR = STREAM ? 1 : NREP;  // (STREAM: one copy — the row loads own the registers)
  uint64_t* const my_rep = NR == 1 ? granules : granules + (me % NR) * REP_STRIDE;

  for (int32_t j = tid; j < (STREAM ? 0 : nrows); j += BS) {  // stage the owned rows into LDS
    const int64_t i = lo + j;
    const double ac = (double)a.alloc_cpu[i], am = (double)a.alloc_mem[i];
    R.ac[j] = ac; R.am[j] = am;
    R.yc[j] = ac != 0.0 ? 1.0 / ac : 0.0;
    R.ym[j] = am != 0.0 ? 1.0 / am : 0.0;
    R.rc[j] = (double)a.req_cpu[i]; R.rm[j] = (double)a.req_mem[i];
    R.zc[j] = (double)a.nz_cpu[i]; R.zm[j] = (double)a.nz_mem[i];
    R.allowed[j] = a.allowed_pods[i]; R.count[j] = a.pod_count[i]; R.fl[j] = a.flags[i];
  }
  // pod descriptors: RING_FILL (1 KiB) per refill, one 16-byte load per lane of wave 1, loaded
  // a whole refill period before they are stored so the load latency never stalls a pod
  // (CACHE: lane l < RING_FILL also carries pod p0 + l's tree class)
  auto ring_load = [&](int64_t p0, uint4& v, int32_t& cl) {
    const int64_t p = p0 + lane / 8;
    if (p < a.end) v = reinterpret_cast<const uint4*>(&a.pods[p])[lane % 8];
    if (CACHE && lane < RING_FILL && p0 + lane < a.end) cl = a.tcls[p0 + lane];
  };
  auto ring_store = [&](int64_t p0, const uint4& v, int32_t cl) {
    const int64_t p = p0 + lane / 8;
    if (p < a.end) reinterpret_cast<uint4*>(&s_pod[p % RING])[lane % 8] = v;
    if (CACHE && lane < RING_FILL && p0 + lane < a.end) s_pcls[(p0 + lane) % RING] = cl;
  };
  uint4 ring_next = make_uint4(0, 0, 0, 0);  // wave 1: descriptors of the next refill
  int32_t ring_next_cl = 0;
  if (wv == 1) {
    uint4 v;
    int32_t cl = 0;
    ring_load(a.first, v, cl);
    ring_load(a.first + RING_FILL, ring_next, ring_next_cl);
    ring_store(a.first, v, cl);
  }
  if (CACHE)
    for (int k = tid; k < a.ncls; k += BS) s_tcl[k] = a.tclass[k];
  if (tid == 0) { s_fix[a.first & 1][0] = -1; s_arr = 0; s_prow[0] = s_prow[1] = -1; }
  uint64_t counter = *a.counter;  // replicated genericScheduler.lastNodeIndex
  __syncthreads();
  // CACHE: a class's inputs as the evaluation reads them (add_* only matter for a commit)
  auto cls_fpod = [&](int k) -> FPod {
    const KsimTreeClass& t = s_tcl[k];
    return FPod{t.rq_c, t.rq_m, t.nz_c, t.nz_m, 0.0, 0.0, t.anyreq, t.be};
  };
  if (CACHE) {  // every (class, owned row) evaluation, once per call
    const int tot = a.ncls * nrows;
    for (int idx = tid; idx < tot; idx += BS) {
      const int k = idx / nrows, j = idx - k * nrows;
      uint32_t rm;
      R.cache[k * chunk + j] = (int16_t)feval(EC, cls_fpod(k), load_frow<false>(R, j), rm);
    }
    __syncthreads();
  }

  auto ptag = [&](int64_t p) -> uint64_t { return (uint64_t)((p - a.first + 1) & 0xFF); };
  // wave-level statistics of NPT evaluations per lane → LDS slot (buf, w)
  auto wave_stats = [&](const int32_t (&e)[NPT], int buf, int w) {
    int32_t v = -1, nf = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      nf += __popcll(__ballot(e[k] >= 0));
      v = e[k] > v ? e[k] : v;
    }
    const int32_t m1 = ksimw::max_i32(v);
    int32_t v2 = -1;
#pragma unroll
    for (int k = 0; k < NPT; ++k) v2 = (e[k] < m1 && e[k] > v2) ? e[k] : v2;
    const int32_t m2 = ksimw::max_i32(v2);
    int32_t c1 = 0, c2 = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const uint64_t bm = m1 < 0 ? 0ull : __ballot(e[k] == m1);
      c1 += __popcll(bm);
      c2 += m2 < 0 ? 0 : __popcll(__ballot(e[k] == m2));
      if (lane == 0) s_bm[buf][k][w - 1] = bm;
    }
    if (lane == 0) {
      s_wst[buf][w - 1][0] = nf; s_wst[buf][w - 1][1] = m1; s_wst[buf][w - 1][2] = c1;
      s_wst[buf][w - 1][3] = m2; s_wst[buf][w - 1][4] = c2;
    }
  };
  // row waves: the last one to finish pod p's statistics merges and publishes them
  auto arrive_publish = [&](int64_t p, int buf) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    int32_t old = 0;
    if (lane == 0) old = atomicAdd(&s_arr, 1);
    old = __builtin_amdgcn_readfirstlane(old);
    if ((old + 1) % RW == 0) {
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
      // lane w < RW holds row wave w's statistics; merged with wave reductions, no branches
      const bool in = lane < RW;
      const int w = in ? lane : 0;
      const int32_t f = in ? s_wst[buf][w][0] : 0;
      const int32_t a1 = s_wst[buf][w][1], n1 = in ? s_wst[buf][w][2] : 0;
      const int32_t a2 = s_wst[buf][w][3], n2 = in ? s_wst[buf][w][4] : 0;
      Top2 t;
      t.f = ksimw::sum_i32(f);
      t.m1 = ksimw::max_i32(n1 ? a1 : -1);
      t.c1 = ksimw::sum_i32((n1 && a1 == t.m1) ? n1 : 0);
      t.m2 = ksimw::max_i32(n1 && a1 < t.m1 ? a1 : (n2 ? a2 : -1));
      t.c2 = ksimw::sum_i32(((n1 && a1 == t.m2) ? n1 : 0) + ((n2 && a2 == t.m2) ? n2 : 0));
      if (t.m2 < 0) t.c2 = 0;
      if (lane == 0) {
        s_wg[buf][0] = t.f; s_wg[buf][1] = t.m1; s_wg[buf][2] = t.c1; s_wg[buf][3] = t.m2; s_wg[buf][4] = t.c2;
        if (NR == 1) store_granule(spec_at(granules, (int)(p % NSLOT), me), gpack(ptag(p), t.f, t.c1, t.m1));
      }
      if (NR > 1 && lane < NR)
        store_granule(spec_at(granules + lane * REP_STRIDE, (int)(p % NSLOT), me), gpack(ptag(p), t.f, t.c1, t.m1));
    }
  };
  // LDS form, control wave: the 64-row segments holding rows at the workgroup maximum of the pod in `buf`
  // (lane t = t-th segment from the top: its bitmask, count, and the matches in segments above
  // it), read before the sweep; the owner turns its rank into a row with a few wave operations
  struct Segs {
    uint64_t m;
    int32_t cnt, base, total;
  };
  auto seg_prepare = [&](int buf) -> Segs {
    constexpr int S = NPT * RW;
    const int32_t M = s_wg[buf][1];
    Segs sg;
    sg.m = 0;
    if (lane < S) {
      const int k = NPT - 1 - lane / RW, w = RW - 1 - lane % RW;
      sg.m = (M >= 0 && s_wst[buf][w][1] == M) ? s_bm[buf][k][w] : 0ull;
    }
    sg.cnt = __popcll(sg.m);
    const int32_t incl = ksimw::prefix_incl_i32(sg.cnt);
    sg.base = incl - sg.cnt;
    sg.total = __builtin_amdgcn_readlane(incl, 63);
    return sg;
  };
  // the rank-th row from the top (-1 if none): the segment holding it, then the bit
  auto seg_select = [&](const Segs& sg, int32_t rank) -> int32_t {
    const uint64_t hs = __ballot(sg.cnt != 0 && rank >= sg.base && rank < sg.base + sg.cnt);
    if (rank >= sg.total || !hs) return -1;
    const int t = __builtin_ctzll(hs);
    const uint64_t ms = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(sg.m >> 32), t) << 32) |
                        (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)sg.m, t);
    const int32_t r = rank - __builtin_amdgcn_readlane(sg.base, t);
    const uint64_t hb = __ballot(((ms >> lane) & 1ull) && __popcll(ms >> lane) - 1 == r);
    if (!hb) return -1;
    const int k = NPT - 1 - t / RW, w = RW - 1 - t % RW;
    return k * RT + w * 64 + __builtin_ctzll(hb);
  };

  // STREAM, control wave: rows at the workgroup maximum of the pod in `buf`, name rank
  // descending, into top_list — so an owner turns its rank into a row with one LDS read (the
  // list is built while the row waves stream, off the critical path; measured faster there
  // than seg_select)
  auto build_top_list = [&](int buf) {
    constexpr int S = NPT * RW;  // lane t = t-th 64-row segment from the top
    const int32_t M = s_wg[buf][1];
    uint64_t m = 0;
    if (lane < S) {
      const int k = NPT - 1 - lane / RW, w = RW - 1 - lane % RW;
      m = (M >= 0 && s_wst[buf][w][1] == M) ? s_bm[buf][k][w] : 0ull;
    }
    const int32_t cnt = __popcll(m);
    const int32_t base = ksimw::prefix_incl_i32(cnt) - cnt;
    uint64_t live = __ballot(cnt != 0);
    while (live) {
      const int t = __builtin_ctzll(live);
      live &= live - 1;
      const uint64_t ms = ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)(m >> 32), t) << 32) |
                          (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)m, t);
      const int32_t b0 = __builtin_amdgcn_readlane(base, t);
      const int k = NPT - 1 - t / RW, w = RW - 1 - t % RW;
      if ((ms >> lane) & 1ull) top_list[b0 + __popcll(ms >> lane) - 1] = k * RT + w * 64 + lane;
    }
  };

  // ---- prologue: evaluations and statistics of the first pod ----
  // reason masks of the evaluations of pod p (A) and p + 1 (B): registers, or (STREAM, up to
  // 9 rows per lane) R.rma in LDS to leave the registers to the row loads
  uint32_t A_rm[STREAM ? 1 : NPT], B_rm[STREAM ? 1 : NPT];
  if (wv > 0) {
    const FPod P0 = load_fpod(s_pod[a.first % RING]);
    int32_t e[NPT];
    int32_t* ev = R.ev + (a.first & 1) * chunk;
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * RT + rt;
      e[k] = -1;
      uint32_t& am = A_rm[STREAM ? 0 : k];
      am = 0;
      if (CACHE) {
        if (j < nrows) e[k] = R.cache[s_pcls[a.first % RING] * chunk + j];
      } else if (j < nrows) {
        e[k] = feval(EC, P0, load_frow<STREAM>(R, j), am);
        if (STREAM) R.rma[(a.first & 1) * chunk + j] = am;
        ev[j] = e[k];
      }
    }
    wave_stats(e, (int)(a.first & 1), wv);
    arrive_publish(a.first, (int)(a.first & 1));
  }
  int X = -1;  // control wave: owner workgroup of the previous pod's node (-1: none)
  int64_t stop_at = a.end;  // first pod not scheduled by this call
  lds_barrier();
#ifdef KSIM_STAMPS
  uint64_t t_prev = __builtin_amdgcn_s_memtime();
  uint64_t tb_prev = t_prev, bw_busy = 0, bw_wait = 0;
#endif

  int64_t last = a.first;  // last pod iterated
  for (int64_t pod = a.first; pod < a.end; ++pod) {
    last = pod;
    const bool has_next = pod + 1 < a.end;
    const int pb = (int)(pod & 1);
    const int nb = (int)((pod + 1) & 1);
    int32_t jsel = -1;      // control wave: row this workgroup commits pod to
    uint64_t stopbit = 0;   // ... and whether that commit leaves the exact float64 range
    FRow jrow;              // STREAM: that row as loaded by the owner
    int32_t e_new = -1;     // STREAM: pod + 1 against the row after pod's commit
    uint32_t m_new = 0;
#ifdef KSIM_STAMPS
    uint64_t o_prev = 0;
#endif

    if (wv == 0) {
      Segs sg{};
      if (STREAM) build_top_list(pb);
      else sg = seg_prepare(pb);
      STAMP(1);
      // ---------------- a. sweep: every workgroup's granule of pod (+ the owner's fix) -------
      const uint64_t tag = ptag(pod);
      const int slot = (int)(pod % NSLOT);
      uint64_t g[MAXB], fx = 0;
      bool ok = false;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
      for (;;) {
#pragma unroll
        for (int j = 0; j < MAXB; ++j) g[j] = load_granule(my_rep + slot * MAXG + j * 64 + lane);
        fx = load_granule(fix_at(my_rep, slot));
        bool mine = X < 0 || gtag(fx) == tag;
#pragma unroll
        for (int j = 0; j < MAXB; ++j) {
          const int b = lane * MAXB + j;
          mine &= (b >= G) || b == X || gtag(g[j]) == tag;
        }
        if (__all(mine)) {
          ok = true;
#pragma unroll
          for (int j = 0; j < MAXB; ++j) g[j] = (lane * MAXB + j == X) ? fx : g[j];
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_LIMIT_TICKS) break;
        __builtin_amdgcn_s_sleep(1);
      }
      STAMP(2);
      PROBE(3);
      // ---------------- b. decide: findNodesThatFit count, max score, selectHost ------------
      // One path for every F > 0: with a single fit node C = 1 and ix = 0 picks it, and only
      // the counter increment differs (generic_scheduler.go:153-156 skips selectHost).
      int32_t f = 0, lm = -1;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) {
        g[j] = (lane * MAXB + j < G) ? g[j] : 0;
        f += gfit(g[j]);
        lm = (gcnt(g[j]) && gscore(g[j]) > lm) ? gscore(g[j]) : lm;
      }
      const int32_t Fl = ksimw::sum_i32(f);
      const int32_t Ml = ksimw::max_i32(lm);
      int32_t bm[MAXB], tot = 0;
#pragma unroll
      for (int j = 0; j < MAXB; ++j) {
        bm[j] = (gcnt(g[j]) && gscore(g[j]) == Ml) ? gcnt(g[j]) : 0;
        tot += bm[j];
      }
      const int32_t pre = ksimw::prefix_incl_i32(tot);
      const int32_t Cl = __builtin_amdgcn_readlane(pre, 63);
      // this rank's (F, M, C); with world > 1, the world's, and the matches on higher ranks
      int32_t F = Fl, M0 = Ml;
      uint32_t C = (uint32_t)Cl;
      int64_t above_r = 0;
      bool stop_any = ok && X >= 0 && gstop(fx);
      if (a.world > 1 && ok) {
        // words (tag:32 | value:32): F, stop:1 | C:31, M — tags run across calls (xtag_base)
        const uint64_t at = (uint64_t)(uint32_t)(a.xtag_base + (uint32_t)(pod - a.first) + 1u) << 32;
        const int aslot = (int)(pod % ANSLOT);
        if (me == 0 && lane < a.world) {
          uint64_t* dst = a.peers[lane] + ((int64_t)aslot * KSIM_MAX_RANKS + a.rank) * 4;
          sys_store(dst, at | (uint32_t)Fl);
          sys_store(dst + 1, at | (stop_any ? 0x80000000ull : 0ull) | (uint32_t)Cl);
          sys_store(dst + 2, at | (uint32_t)Ml);
        }
        const bool rl = lane < a.world;
        const uint64_t* src = a.xchg + ((int64_t)aslot * KSIM_MAX_RANKS + (rl ? lane : 0)) * 4;
        uint64_t w0 = 0, w1 = 0, w2 = 0;
        const uint64_t hi = 0xFFFFFFFF00000000ull;
        for (;;) {
          w0 = sys_load(src);
          w1 = sys_load(src + 1);
          w2 = sys_load(src + 2);
          if (__all(!rl || ((w0 & hi) == at && (w1 & hi) == at && (w2 & hi) == at))) break;
          // the first pod of a call doubles as the start handshake: the peers' kernels may start late
          const uint64_t lim = (pod == a.first) ? a.start_ticks : SPIN_LIMIT_TICKS;
          if (__builtin_amdgcn_s_memrealtime() - t0 > lim) { ok = false; break; }
          __builtin_amdgcn_s_sleep(1);
        }
        const int32_t Fr = rl ? (int32_t)(uint32_t)w0 : 0, Cr = rl ? (int32_t)((uint32_t)w1 & 0x7FFFFFFFu) : 0;
        const int32_t Mr = (rl && Cr) ? (int32_t)(uint32_t)w2 : -1;
        F = ksimw::sum_i32(Fr);
        M0 = ksimw::max_i32(Mr);
        const int32_t Cm = (Cr && Mr == M0) ? Cr : 0;
        const int32_t pr = ksimw::prefix_incl_i32(Cm);
        C = (uint32_t)__builtin_amdgcn_readlane(pr, 63);
        above_r = (int64_t)C - __builtin_amdgcn_readlane(pr, a.rank);  // matches on higher ranks
        stop_any = __any(rl && ((w1 >> 31) & 1));
      }
      const uint32_t Cs = C ? C : 1u;
      const int64_t ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)Cs) : (int64_t)((uint32_t)counter % Cs);
      const int64_t ixl = ix - above_r;  // index among this rank's matches, from the top
      const int64_t above = (int64_t)Cl - pre;  // matches in workgroups of higher lanes
      const bool hit = Ml == M0 && tot > 0 && ixl >= above && ixl < above + tot;
      int32_t found = -1;
      int64_t rr = ixl - above;
#pragma unroll
      for (int j = MAXB - 1; j >= 0; --j) {
        const bool here = found < 0 && rr < bm[j];
        found = here ? lane * MAXB + j : found;
        rr = (found < 0) ? rr - bm[j] : rr;
      }
      const uint64_t hb = __ballot(hit);
      const int src = __builtin_ffsll((long long)hb) - 1;
      const int blk = hb ? __builtin_amdgcn_readlane(found, src) : -1;
      const int rank = hb ? __builtin_amdgcn_readlane((int32_t)rr, src) : 0;
      int mode;
      if (!ok) mode = -1;
      else if (stop_any) mode = -2;  // the previous commit left the exact range
      else if (F == 0) mode = 0;
      else if (hb) mode = blk >= 0 ? 2 : -1;
      else mode = a.world > 1 ? 3 : -1;  // 3: another rank holds the node
      if (mode >= 2 && F > 1) counter += 1;  // generic_scheduler.go:192-195
      if (lane == 0 && mode == -1) atomicOr(a.err, ok ? 2 : 4);
      STAMP(3);
#ifdef KSIM_STAMPS
      o_prev = __builtin_amdgcn_s_memtime();
#endif
      if (mode == 2 && blk == me) {
        // ---------------- c. owner: the rank-th row from the top ----------------
        jsel = STREAM ? (rank < s_wg[pb][2] ? top_list[rank] : -1) : seg_select(sg, rank);
        if (jsel < 0 || jsel >= nrows) {
          jsel = -1;
          mode = -1;
          if (lane == 0) atomicOr(a.err, 2);
        } else if (!STREAM) {
          const ksim_pod& Pp = s_pod[pod % RING];
          stopbit = (R.rc[jsel] + (double)Pp.add_cpu >= EXACT_LIM || R.rm[jsel] + (double)Pp.add_mem >= EXACT_LIM ||
                     R.zc[jsel] + (double)Pp.nz_cpu >= EXACT_LIM || R.zm[jsel] + (double)Pp.nz_mem >= EXACT_LIM)
                        ? (1ull << 55)
                        : 0ull;
        } else if (has_next) {
          // STREAM: the row waves evaluate pod + 1 once per row; the owner evaluates the committed
          // row after pod itself, loading it now while the row waves still stream (a row with a
          // commit still pending from pod - 1 is finished in section d from the streaming lane's copy)
          jrow = load_frow_l2(R, jsel);
          if (jsel != s_prow[nb]) {
            const FRow r2 = plus(jrow, load_fpod(s_pod[pod % RING]));
            e_new = feval(EC, load_fpod(s_pod[(pod + 1) % RING]), r2, m_new);
            stopbit = (r2.rc >= EXACT_LIM || r2.rm >= EXACT_LIM || r2.zc >= EXACT_LIM || r2.zm >= EXACT_LIM) ? (1ull << 55) : 0ull;
          }
        }
        OSTAMP(22);
      }
      if ((mode == 0 || mode == 3) && me == 0 && lane == 0) a.out_node[pod] = mode == 0 ? -1 : -2;
      if (lane == 0) {
        s_mode[pb] = mode;
        s_own[pb] = jsel;
        if (STREAM) {  // the commit itself is applied by the row lane that owns the row
          s_prow[pb] = jsel;
          if (jsel >= 0) {
            const ksim_pod& Pp = s_pod[pod % RING];
            s_pdel[pb][0] = (double)Pp.add_cpu; s_pdel[pb][1] = (double)Pp.add_mem;
            s_pdel[pb][2] = (double)Pp.nz_cpu; s_pdel[pb][3] = (double)Pp.nz_mem;
          }
        }
      }
      X = mode == 2 ? blk : -1;
      STAMP(6);
    } else {
      // STREAM: the deferred commit of pod - 1 to this workgroup's row prow (s_prow[nb]) —
      // the lane that streams the row adds the deltas in registers and stores the row back, so
      // neither the owner's critical path nor a barrier waits on HBM (same-lane program order
      // makes its next load of the row see the store)
      const int32_t prow = STREAM ? s_prow[nb] : -1;
      auto apply_commit = [&](FRow& r, int32_t j) {
        r.rc += s_pdel[nb][0]; r.rm += s_pdel[nb][1]; r.zc += s_pdel[nb][2]; r.zm += s_pdel[nb][3]; r.count += 1;
        R.rc[j] = r.rc; R.rm[j] = r.rm; R.zc[j] = r.zc; R.zm[j] = r.zm; R.count[j] = r.count;
        s_pval[0] = r.rc; s_pval[1] = r.rm; s_pval[2] = r.zc; s_pval[3] = r.zm; s_pcnt = r.count;  // for the owner
      };
      if (STREAM && !has_next && prow >= 0) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * RT + rt;
          if (j == prow) {
            FRow r = load_frow<STREAM>(R, j);
            apply_commit(r, j);
          }
        }
      }
      if (has_next) {
      // ---------------- row waves: evaluate pod + 1, as the rows stand and after pod -----------
      const bool refill = wv == 1 && ((pod - a.first) % RING_FILL) == 0;
      if (refill) ring_store(pod + RING_FILL, ring_next, ring_next_cl);  // loaded a refill period ago
      uint4 rv;
      int32_t rcl = 0;
      if (refill) ring_load(pod + 2 * RING_FILL, rv, rcl);
#ifdef KSIM_STAMPS
      const uint64_t te0 = __builtin_amdgcn_s_memtime();
#endif
      PROBE(4);
      const FPod P = load_fpod(s_pod[pod % RING]);
      const FPod Q = load_fpod(s_pod[(pod + 1) % RING]);
#ifdef KSIM_STAMPS
      uint64_t tw = __builtin_amdgcn_s_memtime();
      if (tid == 64) st_acc[8] += tw - te0;
#define WSTAMP(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); if (tid == 64) st_acc[k] += t_ - tw; tw = t_; } while (0)
#else
#define WSTAMP(k) do { } while (0)
#endif
      // the LDS form evaluates every row twice: as it stands (the speculative statistics every
      // workgroup waits for, published first) and after committing pod (only the owner's
      // correction reads it, so it is computed after the publish); the streaming form evaluates
      // once and its owner evaluates the committed row itself.
      int32_t e[NPT];
      FRow rk[STREAM ? 1 : NPT];
      int32_t* evn = R.ev + nb * chunk;
      if (CACHE) {
        // cached form: pod + 1's statistics are its class's cached evaluations (the rows as they
        // stand), then pod + 1 against "row + pod" only for the rows pod can commit to — the
        // rows at this workgroup's maximum of pod (its owner picks one of them)
        const int16_t* c1 = R.cache + s_pcls[(pod + 1) % RING] * chunk;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * RT + rt;
          e[k] = j < nrows ? (int32_t)c1[j] : -1;
        }
        WSTAMP(9);
        wave_stats(e, nb, wv);
        WSTAMP(10);
        arrive_publish(pod + 1, nb);
        const int32_t M0 = s_wg[pb][1];
        const int16_t* c0 = R.cache + s_pcls[pod % RING] * chunk;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * RT + rt;
          if (M0 >= 0 && j < nrows && (int32_t)c0[j] == M0) {
            uint32_t m2;
            R.ev2[j] = feval(EC, Q, plus(load_frow<false>(R, j), P), m2);
            R.rm2[j] = m2;
          }
        }
      } else {
#pragma unroll
      for (int k = 0; k < NPT; ++k) {
        const int32_t j = k * RT + rt;
        e[k] = -1;
        uint32_t& bm = B_rm[STREAM ? 0 : k];
        bm = 0;
        if (j < nrows) {
          FRow r = load_frow<STREAM>(R, j);
          if (STREAM && j == prow) apply_commit(r, j);
          e[k] = feval(EC, Q, r, bm);
          evn[j] = e[k];
          if (STREAM) {
            R.rma[nb * chunk + j] = bm;
          } else {
            rk[STREAM ? 0 : k] = r;
          }
        }
      }
      WSTAMP(9);
      wave_stats(e, nb, wv);
      WSTAMP(10);
      PROBE(1);
      arrive_publish(pod + 1, nb);
      if (!STREAM) {
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * RT + rt;
          if (j < nrows) {
            uint32_t m2;
            R.ev2[j] = feval(EC, Q, plus(rk[STREAM ? 0 : k], P), m2);
            R.rm2[j] = m2;
          }
        }
      }
      }  // !CACHE
      WSTAMP(11);
#ifdef KSIM_STAMPS
      if (tid == 64) st_acc[5] += __builtin_amdgcn_s_memtime() - te0;
#endif
      if (refill) { ring_next = rv; ring_next_cl = rcl; }
      }
      // STREAM: the wave that applied pod - 1's deferred commit lets its stores reach L2 before
      // the barrier: from the next pod on the owner may read that row (load_frow_l2)
      if (STREAM && prow >= 0 && wv == 1 + (prow % RT) / 64) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
#ifdef KSIM_STAMPS
    const uint64_t tb0 = __builtin_amdgcn_s_memtime();
#endif
    lds_barrier();
#ifdef KSIM_STAMPS
    {  // per wave: time from the last main barrier to this one (busy) and the wait in it
      const uint64_t tb1 = __builtin_amdgcn_s_memtime();
      bw_busy += tb0 - tb_prev;
      bw_wait += tb1 - tb0;
      tb_prev = tb1;
    }
#endif
    STAMP(7);
    const int mode = s_mode[pb];
    if (mode < 0) {  // uniform: every workgroup reaches the same verdict
      if (mode == -2) stop_at = pod;
      break;
    }
    const int32_t own = s_own[pb];

    if (own >= 0) {
      // ---------------- d. owner: correction of pod + 1's statistics, O(1), then the commit ----
      if (wv == 0) {
        OSTAMP(17);
        if (has_next) {
          if (STREAM && jsel == s_prow[nb]) {  // pod - 1's deferred commit hit this row too
            FRow r = jrow;
            r.rc = s_pval[0]; r.rm = s_pval[1]; r.zc = s_pval[2]; r.zm = s_pval[3]; r.count = s_pcnt;
            const FRow r2 = plus(r, load_fpod(s_pod[pod % RING]));
            e_new = feval(EC, load_fpod(s_pod[(pod + 1) % RING]), r2, m_new);
            stopbit = (r2.rc >= EXACT_LIM || r2.rm >= EXACT_LIM || r2.zc >= EXACT_LIM || r2.zm >= EXACT_LIM) ? (1ull << 55) : 0ull;
          }
          if (!STREAM) { e_new = R.ev2[jsel]; m_new = R.rm2[jsel]; }
          // the workgroup's pod + 1 statistics without the committed row's pre-commit
          // evaluation, with its post-commit one (straight-line selects)
          const int32_t e_old = CACHE ? (int32_t)R.cache[s_pcls[(pod + 1) % RING] * chunk + jsel] : R.ev[nb * chunk + jsel];
          const int32_t f0 = s_wg[nb][0], m1 = s_wg[nb][1], c1 = s_wg[nb][2], m2 = s_wg[nb][3], c2 = s_wg[nb][4];
          const bool rem = e_old >= 0, add = e_new >= 0;
          const int32_t c1a = c1 - ((rem && e_old == m1) ? 1 : 0);
          const int32_t mb = c1a ? m1 : (c2 ? m2 : -1), cb = c1a ? c1a : c2;
          const bool up = add && (cb == 0 || e_new > mb), eq = add && !up && e_new == mb;
          const int32_t M = up ? e_new : mb, Cn = up ? 1 : cb + (eq ? 1 : 0);
          const int32_t Ff = f0 - (rem ? 1 : 0) + (add ? 1 : 0);
          PROBE(2);
          if (NR > 1 && lane < NR)
            store_granule(fix_at(granules + lane * REP_STRIDE, (int)((pod + 1) % NSLOT)),
                          gpack(ptag(pod + 1), Ff, Cn, Cn ? M : -1) | stopbit);
          if (lane == 0) {
            if (NR == 1)
              store_granule(fix_at(granules, (int)((pod + 1) % NSLOT)), gpack(ptag(pod + 1), Ff, Cn, Cn ? M : -1) | stopbit);
            s_wg[nb][0] = Ff; s_wg[nb][1] = Cn ? M : -1; s_wg[nb][2] = Cn;
          }
        }
        OSTAMP(18);
        if (CACHE) {
          // the committed row's evaluation for every class (lane k = class k), off the critical
          // path: the next pods' statistics read them after the barrier below
          const FRow r2 = plus(load_frow<false>(R, jsel), load_fpod(s_pod[pod % RING]));
          if (lane < a.ncls) {
            uint32_t rm;
            R.cache[lane * chunk + jsel] = (int16_t)feval(EC, cls_fpod(lane), r2, rm);
          }
        }
        if (lane == 0) {  // commit: NodeInfo.AddPod into the LDS row (STREAM: deferred, s_prow)
          if (!STREAM) {
            const ksim_pod& Pp = s_pod[pod % RING];
            R.rc[jsel] += (double)Pp.add_cpu; R.rm[jsel] += (double)Pp.add_mem;
            R.zc[jsel] += (double)Pp.nz_cpu; R.zm[jsel] += (double)Pp.nz_mem;
            R.count[jsel] += 1;
          }
          if (stopbit) atomicOr(a.err, 8);
          a.out_node[pod] = (int32_t)(a.node_base + lo + jsel);
          if (has_next) {
            R.ev[nb * chunk + jsel] = e_new;
            s_fix[nb][0] = jsel;
            s_fix[nb][1] = (int32_t)m_new;
          } else {
            s_fix[nb][0] = -1;
          }
        }
      }
      lds_barrier();  // uniform (own is workgroup-wide): row waves see the commit
      if (wv == 0 && has_next) {
        // off the critical path: the corrected wave's statistics and bitmasks
        const int w = 1 + (jsel % RT) / 64;
        int32_t e[NPT];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * RT + (w - 1) * 64 + lane;
          e[k] = j < nrows ? (CACHE ? (int32_t)R.cache[s_pcls[(pod + 1) % RING] * chunk + j] : R.ev[nb * chunk + j]) : -1;
        }
        wave_stats(e, nb, w);
        OSTAMP(19);
#ifdef KSIM_STAMPS
        if (lane == 0) atomicAdd((unsigned long long*)&a.dbg[21], 1ull);
#endif
      }
    } else if (wv == 0 && lane == 0) {
      s_fix[nb][0] = -1;
    }

    if (mode == 0 && a.collect && a.out_reasons) {  // FitError: every workgroup adds its reasons
      if (tid < KSIM_NREASONS) s_hist[tid] = 0;
      lds_barrier();
      if (wv > 0) {
        const int32_t fr = s_fix[pb][0];
        const uint32_t fmk = (uint32_t)s_fix[pb][1];
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const int32_t j = k * RT + rt;
          uint32_t rm = (j == fr) ? fmk : !STREAM ? A_rm[STREAM ? 0 : k] : (j < nrows ? R.rma[pb * chunk + j] : 0u);
          if (CACHE) {  // the cached form keeps no reason masks: pod against the rows as they stand
            rm = 0;
            if (j < nrows) (void)feval(EC, load_fpod(s_pod[pod % RING]), load_frow<false>(R, j), rm);
          }
          for (int r = 0; r < KSIM_NREASONS; ++r) {
            const int32_t n = __popcll(__ballot((rm >> r) & 1u));
            if (lane == 0 && n) atomicAdd(&s_hist[r], n);
          }
        }
      }
      lds_barrier();
      if (tid < KSIM_NREASONS && s_hist[tid]) atomicAdd(&a.out_reasons[pod * KSIM_NREASONS + tid], s_hist[tid]);
    }
    STAMP(4);
    if (wv > 0) {
#pragma unroll
      for (int k = 0; k < (STREAM ? 0 : NPT); ++k) A_rm[k] = B_rm[k];
    }
  }

  // the table is authoritative in HBM between calls: write the owned rows back
  __syncthreads();
  if (STREAM) {  // the deferred commit of the last pod iterated (s_prow is -1 after a stop)
    if (tid == 0) {
      const int32_t pr = s_prow[last & 1];
      if (pr >= 0) {
        const double* d = s_pdel[last & 1];
        R.rc[pr] += d[0]; R.rm[pr] += d[1]; R.zc[pr] += d[2]; R.zm[pr] += d[3]; R.count[pr] += 1;
        if (R.rc[pr] >= EXACT_LIM || R.rm[pr] >= EXACT_LIM || R.zc[pr] >= EXACT_LIM || R.zm[pr] >= EXACT_LIM)
          atomicOr(a.err, 8);
      }
    }
    __syncthreads();
  }
  for (int32_t j = tid; j < nrows; j += BS) {
    const int64_t i = lo + j;
    a.req_cpu[i] = (int64_t)R.rc[j]; a.req_mem[i] = (int64_t)R.rm[j];
    a.nz_cpu[i] = (int64_t)R.zc[j]; a.nz_mem[i] = (int64_t)R.zm[j];
    a.pod_count[i] = R.count[j];
  }
  if (me == 0 && tid == 0) {
    *a.counter = counter;
    *a.cursor = stop_at;
  }
#ifdef KSIM_STAMPS
  if (me == 0 && lane == 0) {
    atomicAdd((unsigned long long*)&a.dbg[32 + wv], bw_busy);
    atomicAdd((unsigned long long*)&a.dbg[40 + wv], bw_wait);
  }
  if (me == 0 && tid == 0)
    for (int k = 0; k < 16; ++k) a.dbg[k] += (k == 5 || (k >= 8 && k <= 11)) ? 0 : st_acc[k];
  if (me == 0 && tid == 64)
    for (int k : {5, 8, 9, 10, 11}) a.dbg[k] += st_acc[k];
#endif
}

// ---------------------------------------------------------------------------------------
static constexpr int PF_LDS_BUDGET = 150 * 1024;

// Same grid rule as ksim_persistent_config (one workgroup per CU, <= 256, >= 64 rows each).
// stream = 0: the rows live in LDS (up to ~400k nodes per device); stream = 1: the rows
// stream from the HBM float64 image every pod and only the evaluations stay in LDS (up to
// 9 rows per row thread: ~1M nodes per device).
extern "C" int ksim_pfast_config(int64_t n, int max_grid, int stream, int* grid, int* lds_rows) {
  int dev = 0;
  hipDeviceProp_t p;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  int g = p.multiProcessorCount;
  if (max_grid > 0 && g > max_grid) g = max_grid;
  if (g <= 0 || n <= 0) return 0;
  if (g > MAXG) g = MAXG;
  if (n < (int64_t)g * 64) g = (int)((n + 63) / 64);
  if (g < 1) g = 1;
  const int64_t chunk = (n + g - 1) / g;
  if (stream) {
    if (chunk * LDS_ROW_BYTES_STREAM > PF_LDS_BUDGET || chunk > 9 * RT) return 0;
  } else if (chunk * LDS_ROW_BYTES > PF_LDS_BUDGET || chunk > 4 * RT) {
    return 0;
  }
  *grid = g;
  *lds_rows = (int)chunk;
  return 1;
}

extern "C" size_t ksim_pfast_granule_bytes(void) { return (size_t)NREP * REP_STRIDE * sizeof(uint64_t); }

// the fast kernel's aggregate slots, then the launch form's (KSIM_LX_*) at ksim_shard_lx_offset()
extern "C" size_t ksim_shard_lx_offset(void) { return (size_t)ANSLOT * KSIM_MAX_RANKS * 4; }  // in words
extern "C" size_t ksim_shard_xchg_bytes(void) {
  return (ksim_shard_lx_offset() + (size_t)KSIM_LX_SLOTS * KSIM_MAX_RANKS * (KSIM_LX_REC + KSIM_PX_REC)) *
         sizeof(uint64_t);
}

// float64 image of the node table for the streaming form: one pass over the int64 columns
// (48 B read, 48 B written per node) before each streaming call.
__global__ __launch_bounds__(256) void ksim_pstream_prepare_kernel(const int64_t* __restrict__ ac, const int64_t* __restrict__ am,
                                                                    const int64_t* __restrict__ rc, const int64_t* __restrict__ rm,
                                                                    const int64_t* __restrict__ zc, const int64_t* __restrict__ zm,
                                                                    int64_t n, double* __restrict__ m) {
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const double dac = (double)ac[i], dam = (double)am[i];
    m[i] = dac;
    m[n + i] = dam;
    m[2 * n + i] = (double)rc[i];
    m[3 * n + i] = (double)rm[i];
    m[4 * n + i] = (double)zc[i];
    m[5 * n + i] = (double)zm[i];
  }
}

extern "C" hipError_t ksim_pstream_prepare(const KsimCtx* c, double* mirror, hipStream_t s) {
  const int pg = (int)std::min<int64_t>((c->n + 255) / 256, 4096);
  hipLaunchKernelGGL(ksim_pstream_prepare_kernel, dim3(pg), dim3(256), 0, s, c->alloc_cpu, c->alloc_mem,
                     (const int64_t*)c->req_cpu, (const int64_t*)c->req_mem, (const int64_t*)c->nz_cpu,
                     (const int64_t*)c->nz_mem, c->n, mirror);
  return hipGetLastError();
}

// LDS bytes of the cached form's evaluations ([ncls][lds_rows] int16), 0 when it does not fit
// beside the rows; the cached form needs every map score below 2^15 (host-checked).
extern "C" size_t ksim_pfast_cache_bytes(int lds_rows, int ncls) {
  if (ncls <= 0 || ncls > KSIM_TREE_MAX_CLASSES || lds_rows <= 0) return 0;
  const size_t b = ((size_t)ncls * lds_rows * 2 + 15) & ~(size_t)15;
  return (size_t)lds_rows * LDS_ROW_BYTES + b <= (size_t)PF_LDS_BUDGET ? b : 0;
}

extern "C" hipError_t ksim_launch_pfast(const KsimCtx* c, uint64_t* granules, int grid, int lds_rows, double* mirror,
                                        const KsimShard* sh, const int32_t* tcls, const KsimTreeClass* tclass, int ncls,
                                        hipStream_t s) {
  PfArgs a;
  a.tcls = tcls; a.tclass = tclass; a.ncls = ncls;
  a.rank = sh->rank; a.world = sh->world; a.node_base = sh->node_base; a.xtag_base = sh->xtag_base;
  a.xchg = sh->xchg;
  for (int r = 0; r < KSIM_MAX_RANKS; ++r) a.peers[r] = sh->peers[r];
  a.start_ticks = sh->start_ticks > SPIN_LIMIT_TICKS ? sh->start_ticks : SPIN_LIMIT_TICKS;
  a.n = c->n; a.chunk = c->chunk; a.first = c->first; a.end = c->end;
  a.alloc_cpu = c->alloc_cpu; a.alloc_mem = c->alloc_mem; a.allowed_pods = c->allowed_pods; a.flags = c->flags;
  a.req_cpu = c->req_cpu; a.req_mem = c->req_mem; a.nz_cpu = c->nz_cpu; a.nz_mem = c->nz_mem;
  a.pod_count = c->pod_count; a.pods = c->pods; a.counter = c->counter; a.cursor = c->cursor;
  a.out_node = c->out_node; a.out_reasons = c->out_reasons; a.err = c->err; a.dbg = c->dbg; a.granules = granules;
  a.preds = c->preds; a.no_prio = c->no_prio; a.collect = c->collect;
  a.wl = (int32_t)c->w[KSIM_W_LEAST_REQUESTED]; a.wm = (int32_t)c->w[KSIM_W_MOST_REQUESTED];
  a.wb = (int32_t)c->w[KSIM_W_BALANCED];
  a.mirror = mirror;
  // every workgroup resident at once (the kernel spins on its peers), then the launch
#define KSIM_PFC(R, S, C, L)                                                           \
  do {                                                                                 \
    hipError_t e_ = ksim_check_coresident(ksim_pfast_kernel<R, S, C>, grid, BS, L);    \
    if (e_ != hipSuccess) return e_;                                                   \
    hipLaunchKernelGGL((ksim_pfast_kernel<R, S, C>), dim3(grid), dim3(BS), L, s, a);   \
  } while (0)
#define KSIM_PF(R, S, L) KSIM_PFC(R, S, false, L)
  if (mirror) {  // streaming form (image prepared by ksim_pstream_prepare on the same stream)
    const size_t lds = (size_t)lds_rows * LDS_ROW_BYTES_STREAM;
    if (lds_rows <= RT) KSIM_PF(1, true, lds);
    else if (lds_rows <= 2 * RT) KSIM_PF(2, true, lds);
    else if (lds_rows <= 4 * RT) KSIM_PF(4, true, lds);
    else KSIM_PF(9, true, lds);
    return hipGetLastError();
  }
  const size_t cb = ncls > 0 ? ksim_pfast_cache_bytes(lds_rows, ncls) : 0;
  if (ncls > 0 && !cb) return hipErrorInvalidValue;
  const size_t lds = (size_t)lds_rows * LDS_ROW_BYTES + cb;
  if (cb) {  // cached form
    if (lds_rows <= RT) KSIM_PFC(1, false, true, lds);
    else if (lds_rows <= 2 * RT) KSIM_PFC(2, false, true, lds);
    else KSIM_PFC(4, false, true, lds);
    return hipGetLastError();
  }
  if (lds_rows <= RT) KSIM_PF(1, false, lds);
  else if (lds_rows <= 2 * RT) KSIM_PF(2, false, lds);
  else KSIM_PF(4, false, lds);
#undef KSIM_PF
#undef KSIM_PFC
  return hipGetLastError();
}
