// ksim_persistent.hip — persistent-kernel mode (KSIM_MODE_PERSISTENT).
//
// One launch walks the whole pod queue.  Workgroup b owns the contiguous name-rank range
// [b*chunk, (b+1)*chunk) of the node table and keeps those rows in LDS for the whole launch
// (only the owner of a node reads or writes it, so node state needs no cross-workgroup
// coherence).  Each 512-thread workgroup splits into one CONTROL wave and seven ROW waves:
//
//   control wave (wave 0)                      row waves (1..7)
//   a. publish the partial of pod p            b. evaluate pod p+1 against the rows,
//      (tagged 8-byte granules)                   speculatively (as if p's winner were not
//   c. sweep every workgroup's granules of p,     in this range — true for all workgroups
//      decide (findNodesThatFit →                 but one); wave-level (max, count) into LDS
//      PrioritizeNodes → selectHost,
//      core/generic_scheduler.go:112-198)
//   d. owner of p's winner only: pick the exact row from p's entries in LDS, commit it
//      (NodeInfo.AddPod) and publish the correction of its p+1 partial — O(1): the row waves
//      evaluated p+1 on every row twice (ev: as is; ev2: with p committed to that row, the
//      "dual hypothesis") and kept each reduce class's top two (value, count), so replacing
//      one row's entry needs no re-evaluation and no re-reduction.
//   ------------------------------- barrier -------------------------------
//
// so the full-table evaluation of the next pod runs concurrently with the exchange, and the
// critical path per pod is sweep → decide → (owner) select + commit + O(1) correction.
// lastNodeIndex is replicated in every workgroup's control wave.  Granules are
// double-buffered by pod parity with an 8-bit pod tag: a workgroup that publishes pod p has
// seen every workgroup's pod p-1 partial, so nobody still reads the p-2 slot it overwrites.
// Every spin is bounded (2 s) and reports through the error word.  Pod descriptors stream
// through a 4-slot LDS ring two pods ahead, so no 128-byte descriptor is pinned in SGPRs.
//
// Granule q of a workgroup: tag:8 | fit:12 (q = 0 only) | count:12 | score:32 (class q max,
// -1 = no fit node of that class).  Scores < 2^31 and chunks <= 4095 rows (host checks).
// Sweep lane l reads workgroups [l*MAXB, l*MAXB+MAXB): name-rank order is lane-major, so the
// matches above a workgroup are one DPP prefix sum away.
#include <cstdlib>
#include <type_traits>

#include "ksim_fast.h"
#include "ksim_wave.h"

namespace {

constexpr int GR = KSIM_MAX_RCLASS;                  // granules per workgroup per slot
constexpr int MAXB = 4;                              // most workgroups per sweep lane (grid <= 256)
constexpr int RING = 16;                             // pod-descriptor ring slots in LDS
constexpr int RING_FILL = 8;                         // descriptors fetched per refill
constexpr uint64_t SPIN_LIMIT_TICKS = 200000000ull;  // s_memrealtime ticks at 100 MHz = 2 s
constexpr int NSLOT = 4;                             // granule slots (pod mod NSLOT)
constexpr int MAXG = 64 * MAXB;                      // workgroups a slot is sized for
constexpr int KF = 4;                                // reduce classes polled per round trip

typedef __attribute__((address_space(1))) uint64_t gu64;

__device__ __forceinline__ void store_granule(uint64_t* g, uint64_t v) {
  __hip_atomic_store((gu64*)g, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ uint64_t load_granule(const uint64_t* g) {
  return __hip_atomic_load((gu64*)g, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
// speculative partial of workgroup b for the pod in `slot`, and the previous owner's correction
// Dense layout [slot][q][pos(b)]: one poll of class 0 touches 2 KiB (16 lines) instead of a
// line per workgroup.  pos(b) = (b % MAXB) * 64 + b / MAXB, so the sweep's j-th load of lane l
// (position j * 64 + l, coalesced across the wave) is workgroup l * MAXB + j.
// MB: workgroups per sweep lane of the kernel instance (1 for grids of <= 64, else MAXB)
template <int MB>
__device__ __forceinline__ uint64_t* spec_at(uint64_t* gr, int slot, int b, int q) {
  return gr + ((int64_t)slot * GR + q) * MAXG + (b % MB) * 64 + b / MB;
}
__device__ __forceinline__ uint64_t* fix_at(uint64_t* gr, int slot, int q) {
  return gr + (int64_t)NSLOT * MAXG * GR + (int64_t)slot * GR + q;
}
template <int MB>
__device__ __forceinline__ uint64_t* gran_at(uint64_t* gr, int slot, int b, int q, int X) {
  return b == X ? fix_at(gr, slot, q) : spec_at<MB>(gr, slot, b, q);
}
__device__ __forceinline__ uint32_t gtag(uint64_t v) { return (uint32_t)(v >> 56); }
__device__ __forceinline__ int32_t gfit(uint64_t v) { return (int32_t)((v >> 44) & 0xFFF); }
__device__ __forceinline__ int32_t gcnt(uint64_t v) { return (int32_t)((v >> 32) & 0xFFF); }
__device__ __forceinline__ int32_t gscore(uint64_t v) { return (int32_t)(uint32_t)v; }

// critical-path probe (diagnostic builds, -DKSIM_PROBE=k): a 512-cycle delay at point k; the
// per-pod time grows by the delay only where k sits on the critical path
#ifdef KSIM_PROBE
#define PROBE(k) do { if (KSIM_PROBE == (k)) __builtin_amdgcn_s_sleep(8); } while (0)
#define PROBE_IF(k, cond) do { if (KSIM_PROBE == (k) && (cond)) __builtin_amdgcn_s_sleep(8); } while (0)
#else
#define PROBE(k) do { } while (0)
#define PROBE_IF(k, cond) do { } while (0)
#endif

#ifdef KSIM_STAMPS
// phase cycle sums kept in registers of block 0's control wave, written once at the end
#define STAMP(k)                                         \
  do {                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();   \
    st_acc[k] += t_ - t_prev;                           \
    t_prev = t_;                                        \
  } while (0)
// owner-side phase durations, summed over whichever workgroup owns each pod
#define OSTAMP(k)                                                        \
  do {                                                                   \
    const uint64_t t_ = __builtin_amdgcn_s_memtime();                   \
    if (lane == 0) atomicAdd((unsigned long long*)&c.dbg[k], t_ - o_prev); \
    o_prev = t_;                                                         \
  } while (0)
#else
#define OSTAMP(k) \
  do {            \
  } while (0)
#define STAMP(k) \
  do {           \
  } while (0)
#endif

// Packed evaluation of one row for one pod: -1 = does not fit, else class:4 | score:27
// (map scores < 2^27, host-checked; reduce classes < 16).
constexpr int EV_SHIFT = 27;
__device__ __forceinline__ int32_t ev_pack(bool fit, int32_t cl, int32_t sc) { return fit ? (cl << EV_SHIFT) | sc : -1; }
__device__ __forceinline__ int32_t ev_cls(int32_t e) { return e >> EV_SHIFT; }
__device__ __forceinline__ int32_t ev_score(int32_t e) { return e & ((1 << EV_SHIFT) - 1); }

// LDS image of one owned row, array-of-structs: every field is an immediate offset from one
// per-lane address (row * 116 B), so the evaluation holds no per-column base addresses in
// scalar registers; the 29-dword stride keeps a wave's same-field accesses on distinct banks.
struct __attribute__((packed, aligned(4))) LRow {
  int64_t ac, am, rc, rm, zc, zm;
  double dac, dam;  // alloc as float64 (derived, for the fast path)
  int32_t allowed, count;
  uint32_t fl;
  int32_t ls, ts;    // label-set / taint-set id of the row
  int32_t ev[2];     // per pod parity: packed evaluation of the row (ev_pack)
  int32_t ev2[2];    // per pod parity: the evaluation with the previous pod committed to the row
  uint32_t rm1[2];   // reason mask of ev
  uint32_t rm2[2];   // ... and of ev2
};

constexpr int LDS_ROW_BYTES = (int)sizeof(LRow);  // 116
static_assert(sizeof(LRow) == 116, "LRow layout");

extern __shared__ __attribute__((aligned(16))) char ksim_smem[];  // dynamic LDS: the row image

}  // namespace

// Dynamic-LDS plan of a workgroup beyond the rows (host-computed in ksim_launch_persistent):
// the rows' host ports and the pod-class tables are staged too when they fit, so the row waves
// — the CU that polls the exchange — issue no global loads while evaluating (a loaded consumer
// CU pays 2.5-2.9 us per hand-off instead of 1.1, MI355X_MICROARCH.md handoff-1to1).
struct PLayout {
  int32_t ps;          // port slots staged per row (0: ports read from HBM)
  int32_t tables;      // 1: sel_ok / taint_ok / noexec_ok / tt_class / na_class staged
  int32_t off_pc, off_pk, off_sel, off_tok, off_nok, off_ttc, off_nac;  // byte offsets in ksim_smem
  int32_t off_ttv, off_nav;  // [C][val_w] reduce-class map values (int64)
  int32_t off_nad;           // [C][val_w] NodePreferAvoidPods addends (int64), staged when present
  // [C][rows] uint16 per (pod class, owned row), built at launch from the class tables: bit 0 the
  // selector does not match, bit 1 / 2 a NoSchedule+NoExecute / NoExecute taint is not
  // tolerated, bits 4-7 / 8-11 the TaintToleration / NodeAffinity reduce class — one LDS load
  // beside the row's own instead of two dependent table lookups per evaluation (0: not staged)
  int32_t off_st;
};

namespace {

// Commit of the columns that stay in HBM (gpu, ephemeral, scalars, ports) and of the
// over-commit bits (node_info.go:318-341, utils.go:45-60).  Single thread of the owner.
__device__ __noinline__ uint32_t commit_side(const KsimCtx* __restrict__ cg, const ksim_pod* Pp, int64_t w, uint32_t fl,
                                             int32_t ports) {
  const KsimCtx& c = *cg;
  const ksim_pod& P = *Pp;
  const int64_t g = c.req_gpu[w] + P.add_gpu;
  const int64_t e = c.req_eph[w] + P.add_eph;
  c.req_gpu[w] = g;
  c.req_eph[w] = e;
  fl &= ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
  if (c.alloc_gpu[w] < g) fl |= KSIM_N_GPU_OVER;
  if (c.alloc_eph[w] < e) fl |= KSIM_N_EPH_OVER;
  for (int32_t s = 0; s < P.scalar_cnt; ++s) {
    const ksim_scalar_req q = c.pod_scalars[P.scalar_off + s];
    c.req_scalar[(int64_t)q.col * c.n + w] += q.add;
  }
  for (int32_t k = 0; ports && k < P.port_cnt; ++k) {
    const uint64_t key = c.pod_ports[P.port_off + k];
    const int32_t cnt = c.port_count[w];
    bool dup = false;
    for (int32_t s = 0; s < cnt; ++s)
      if (c.ports[(int64_t)s * c.n + w] == key) { dup = true; break; }
    if (dup) continue;
    if (cnt >= c.port_slots) { atomicOr(c.err, 1); continue; }
    c.ports[(int64_t)cnt * c.n + w] = key;
    c.port_count[w] = cnt + 1;
  }
  return fl;
}

// HostPortInfo.Add of the pod's ports on row j when the rows' ports are staged in LDS: the set
// is read from LDS, new keys written to LDS and HBM (stores only, nothing waits on HBM).
__device__ __noinline__ void commit_ports_lds(const KsimCtx* __restrict__ cg, const ksim_pod* Pp, int64_t w, int32_t j,
                                              int32_t rows, int32_t off_pc, int32_t off_pk) {
  const KsimCtx& c = *cg;
  const ksim_pod& P = *Pp;
  int32_t* pc = reinterpret_cast<int32_t*>(ksim_smem + off_pc);
  uint64_t* pk = reinterpret_cast<uint64_t*>(ksim_smem + off_pk);
  int32_t cnt = pc[j];
  for (int32_t k = 0; k < P.port_cnt; ++k) {
    const uint64_t key = c.pod_ports[P.port_off + k];
    bool dup = false;
    for (int32_t s = 0; s < cnt; ++s)
      if (pk[s * rows + j] == key) { dup = true; break; }
    if (dup) continue;
    if (cnt >= c.port_slots) { atomicOr(c.err, 1); continue; }
    pk[cnt * rows + j] = key;
    c.ports[(int64_t)cnt * c.n + w] = key;
    cnt += 1;
  }
  pc[j] = cnt;
  c.port_count[w] = cnt;
}

// Total score of reduce class q once the per-class maxima over the filtered set are known
// (NormalizeReduce, priorities/reduce.go:29-64; weighted sum generic_scheduler.go:632-639).
// tv / av: the class's TaintToleration / NodeAffinity map values (prefetched per pod).
__device__ __forceinline__ int64_t class_total(const KsimCtx& c, int64_t tv, int64_t av, int64_t ad, int64_t base,
                                               int64_t mxT, int64_t mxA) {
  uint64_t t = (uint64_t)base + (uint64_t)ad;  // ad: NodePreferAvoidPods' weighted score of the class
  if (c.w[KSIM_W_TAINT_TOLERATION]) t += (uint64_t)c.w[KSIM_W_TAINT_TOLERATION] * (uint64_t)ksim_norm(tv, mxT, true);
  if (c.w[KSIM_W_NODE_AFFINITY]) t += (uint64_t)c.w[KSIM_W_NODE_AFFINITY] * (uint64_t)ksim_norm(av, mxA, false);
  return (int64_t)t;
}

// wave-wide maximum of a 64-bit value: the DPP int32 reduction when every lane's value fits
// (the common case: counts, weights, scores), else a shuffle tree (ds_bpermute, ~10x slower)
__device__ __forceinline__ int64_t wave_max_i64(int64_t v) {
  if (__all(v >= INT32_MIN && v <= INT32_MAX)) return ksimw::max_i32((int32_t)v);
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const int64_t t = __shfl_xor(v, o, 64);
    v = t > v ? t : v;
  }
  return v;
}

// 64-bit value of lane q (wave-uniform q)
__device__ __forceinline__ int64_t readlane64(int64_t v, int q) {
  return (int64_t)(((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)((uint64_t)v >> 32), q) << 32) |
                   (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int32_t)v, q));
}

// A committed pod's change to a row (NodeInfo.AddPod of the resource-only part): the dual
// hypothesis evaluates the next pod on row + delta.  pp: the two pods' host ports conflict.
struct RowDelta {
  int64_t c, m, zc, zm;
  int32_t n, pp;
  int64_t g, e;  // gpu / ephemeral adds (the over-commit bits are re-derived from HBM)
};

}  // namespace

// The uniform inputs of one pod's evaluation, read once per pod from the LDS ring into
// registers (the per-row evaluation then touches LDS only for the row and its table bits).
struct PodView {
  int64_t rq_c, rq_m, rq_g, rq_e, nz_c, nz_m;
  uint32_t flags;
  int32_t host, cls, k1, k2;
  int32_t port_cnt, port_off, scalar_off, scalar_cnt;
  bool fast;  // resource-only (ksim_is_fast_pod)
};

// Pin a wave-uniform value into VGPRs: the kernel's scalar file is full (both roles share one
// allocation), so uniform per-pod inputs held in SGPRs get spilled to VGPR lanes and reloaded
// with a v_readlane at every use inside the row evaluation; an asm operand the compiler must
// treat as divergent keeps them in vector registers instead.
template <class T>
__device__ __forceinline__ void to_vgpr(T& x) {
  asm volatile("" : "+v"(x));
}

__device__ __forceinline__ void to_vgpr(bool& x) {
  int32_t t = x;
  asm volatile("" : "+v"(t));
  x = t != 0;
}

// The descriptor in LDS → PodView with eight 16-byte reads issued together.
__device__ __forceinline__ PodView pod_view_lds(const ksim_pod* Pl);

__device__ __forceinline__ PodView pod_view(const ksim_pod& P) {
  PodView V;
  V.rq_c = P.req_cpu; V.rq_m = P.req_mem; V.rq_g = P.req_gpu; V.rq_e = P.req_eph;
  V.nz_c = P.nz_cpu; V.nz_m = P.nz_mem;
  V.flags = P.flags; V.host = P.host; V.cls = P.cls; V.k1 = P.reserved[0]; V.k2 = P.reserved[1];
  V.port_cnt = P.port_cnt; V.port_off = P.port_off; V.scalar_off = P.scalar_off; V.scalar_cnt = P.scalar_cnt;
  V.fast = ksim_is_fast_pod(P, V.k1 * V.k2);
  return V;
}

__device__ __forceinline__ PodView pod_view_lds(const ksim_pod* Pl) {
  const uint4* w = reinterpret_cast<const uint4*>(Pl);
  uint4 a[sizeof(ksim_pod) / 16];
#pragma unroll
  for (int k = 0; k < (int)(sizeof(ksim_pod) / 16); ++k) a[k] = w[k];
  ksim_pod P;
  __builtin_memcpy(&P, a, sizeof P);
  return pod_view(P);
}

template <int BS, int NPT, int MB>
__global__ __launch_bounds__(BS) void ksim_persistent_kernel(KsimCtx c, const KsimCtx* __restrict__ cg,
                                                             uint64_t* granules, PLayout L) {
  constexpr int NW = BS / 64;
  constexpr int RT = BS - 64;          // row threads
  constexpr int SPLIT_ROWS = 192;       // dual-hypothesis split: ev on the first waves, ev2 on the next
  constexpr int PPK = 4;                 // host-port keys staged per pod descriptor
  __shared__ int32_t s_mx[2][NW][KSIM_MAX_RCLASS];   // per row wave, double-buffered by pod parity:
  __shared__ int32_t s_cnt[2][NW][KSIM_MAX_RCLASS];  // per reduce class the top value and its count,
  __shared__ int32_t s_mx2[2][NW][KSIM_MAX_RCLASS];  // the second value and its count
  __shared__ int32_t s_cnt2[2][NW][KSIM_MAX_RCLASS];
  __shared__ int32_t s_fit[2][NW];
  __shared__ int4 s_top[2][KSIM_MAX_RCLASS];  // the workgroup's (top, count, second, count) per class
  __shared__ int32_t s_F[2];                  // ... its fit rows
  __shared__ int32_t s_done[2];               // tag of the pod whose workgroup stats are complete
  __shared__ int32_t s_ev2[2];                // 1: ev2 was evaluated for that pod
  // one row per row thread (NPT == 1): per row wave and class, the rows at the wave's top value
  // (bit l = row (w-1)*64 + l), so the owner's selectHost pick needs no scan of the entries;
  // s_mok: the masks are exact for that pod (an owner correction that empties a wave's top
  // clears it, and the owner then scans)
  __shared__ uint64_t s_msk[2][NW][KSIM_MAX_RCLASS];
  __shared__ int32_t s_mok[2];
  __shared__ uint64_t s_gq[KSIM_MAX_RCLASS - 1 - KF][MAXG];  // control wave: granules of classes > KF (by b)
  __shared__ int32_t s_dec;    // pods decided and committed (control wave → row waves)
  __shared__ int32_t s_abort;  // the control wave stopped on an error
  __shared__ int32_t s_arr[2];  // row-wave arrivals per pod parity (the last one of a pod publishes)
  __shared__ __attribute__((aligned(16))) ksim_pod s_pod[RING];
  __shared__ uint64_t s_ppk[RING][PPK];  // the ring's pods' host-port keys (pods with <= PPK ports)
#ifdef KSIM_STAMPS
  uint64_t st_acc[16] = {};
  uint64_t ev_acc[4] = {};  // row wave 1: pod view, evaluation, read-back (tid 64 of block 0)
  uint64_t wait_acc = 0;    // row wave 1: waiting for the control wave (s_dec)
#endif

  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const int rt = tid - 64;  // row-thread index (row waves only)
  const int G = gridDim.x;
  const int64_t chunk = c.chunk;
  const int64_t lo = (int64_t)blockIdx.x * chunk;
  const int64_t hi = (lo + chunk < c.n) ? lo + chunk : c.n;
  const int32_t nrows = (int32_t)(hi - lo);
  LRow* const RW = reinterpret_cast<LRow*>(ksim_smem);
  const uint32_t preds = c.preds;
  const int64_t wl = c.w[KSIM_W_LEAST_REQUESTED], wmr = c.w[KSIM_W_MOST_REQUESTED], wb = c.w[KSIM_W_BALANCED];
  const bool no_prio = c.no_prio != 0;
  // dual hypothesis layout: split (ev and ev2 on disjoint waves) when the rows fit both halves
  const bool split = NPT == 1 && nrows <= SPLIT_ROWS;
  // row waves with rows to evaluate (split: the ev waves from row thread 0, the ev2 waves from
  // `half`); the others sit the pod loop out — they would only add arrivals and LDS traffic
  auto active = [&](int w) -> bool {
    if (w == 1) return true;  // refills the pod ring; publishes (empty) partials of a range with no rows
    const int r0 = (w - 1) * 64;
    if (!split) return r0 < nrows || NPT > 1;
    const int hf = 64 * ((nrows + 63) / 64);
    return r0 < nrows || (r0 >= hf && r0 - hf < nrows);
  };
  int nact = 0;
  for (int w = 1; w < NW; ++w) nact += active(w) ? 1 : 0;

  for (int32_t j = tid; j < nrows; j += BS) {  // stage the owned rows into LDS
    const int64_t i = lo + j;
    const int64_t ac = c.alloc_cpu[i], am = c.alloc_mem[i];
    RW[j].ac = ac; RW[j].am = am;
    RW[j].dac = (double)ac;
    RW[j].dam = (double)am;
    RW[j].rc = c.req_cpu[i]; RW[j].rm = c.req_mem[i];
    RW[j].zc = c.nz_cpu[i]; RW[j].zm = c.nz_mem[i];
    RW[j].allowed = c.allowed_pods[i]; RW[j].count = c.pod_count[i]; RW[j].fl = c.flags[i];
    RW[j].ls = c.label_set[i]; RW[j].ts = c.taint_set[i];
    if (L.ps) {  // the rows' host ports (HostPortInfo), slot-major like the HBM column
      reinterpret_cast<int32_t*>(ksim_smem + L.off_pc)[j] = c.port_count[i];
      for (int32_t q = 0; q < L.ps; ++q)
        reinterpret_cast<uint64_t*>(ksim_smem + L.off_pk)[q * chunk + j] = c.ports[(int64_t)q * c.n + i];
    }
  }
  if (L.tables) {  // the pod-class tables (selector / toleration bits, reduce-class bytes)
    const int32_t C = c.n_classes_dev;
    for (int32_t k = tid; k < C * c.lwords; k += BS) reinterpret_cast<uint32_t*>(ksim_smem + L.off_sel)[k] = c.sel_ok[k];
    for (int32_t k = tid; k < C * c.twords; k += BS) {
      reinterpret_cast<uint32_t*>(ksim_smem + L.off_tok)[k] = c.taint_ok[k];
      reinterpret_cast<uint32_t*>(ksim_smem + L.off_nok)[k] = c.noexec_ok[k];
    }
    for (int32_t k = tid; k < C * c.n_taint_sets; k += BS) (ksim_smem + L.off_ttc)[k] = (char)c.tt_class[k];
    for (int32_t k = tid; k < C * c.n_label_sets; k += BS) (ksim_smem + L.off_nac)[k] = (char)c.na_class[k];
    for (int32_t k = tid; k < C * c.val_w; k += BS) {
      reinterpret_cast<int64_t*>(ksim_smem + L.off_ttv)[k] = c.tt_val[k];
      reinterpret_cast<int64_t*>(ksim_smem + L.off_nav)[k] = c.na_val[k];
      if (c.na_add) reinterpret_cast<int64_t*>(ksim_smem + L.off_nad)[k] = c.na_add[k];
    }
  }
  if (L.off_st) {  // static per-(class, row) bits; the staged tables are read back after the barrier
    __syncthreads();
    const int32_t C = c.n_classes_dev;
    uint16_t* st = reinterpret_cast<uint16_t*>(ksim_smem + L.off_st);
    for (int32_t k = tid; k < C * nrows; k += BS) {
      const int32_t cls = k / nrows, j = k - cls * nrows;
      const int32_t ls = RW[j].ls, ts = RW[j].ts;
      const uint32_t ws = reinterpret_cast<const uint32_t*>(ksim_smem + L.off_sel)[(int64_t)cls * c.lwords + (ls >> 5)];
      const uint32_t wt = reinterpret_cast<const uint32_t*>(ksim_smem + L.off_tok)[(int64_t)cls * c.twords + (ts >> 5)];
      const uint32_t wn = reinterpret_cast<const uint32_t*>(ksim_smem + L.off_nok)[(int64_t)cls * c.twords + (ts >> 5)];
      const uint32_t a = (uint8_t)(ksim_smem + L.off_ttc)[(int64_t)cls * c.n_taint_sets + ts];
      const uint32_t b = (uint8_t)(ksim_smem + L.off_nac)[(int64_t)cls * c.n_label_sets + ls];
      st[(int64_t)cls * chunk + j] = (uint16_t)((((ws >> (ls & 31)) & 1u) ^ 1u) | ((((wt >> (ts & 31)) & 1u) ^ 1u) << 1) |
                                                ((((wn >> (ts & 31)) & 1u) ^ 1u) << 2) | ((a & 15u) << 4) | ((b & 15u) << 8));
    }
  }
  // pod ring: RING_FILL descriptors (1 KiB) per refill, one 16-byte load per lane of wave 1, then
  // their host-port keys (lane 4s+k: key k of the refill's pod s).  The reduce-class counts k1
  // (TaintToleration) / k2 (NodeAffinity) ride in each queued descriptor's reserved[0..1]
  // (written by the library, ksim_launch_pod_k).
  auto ring_load = [&](int64_t p0, uint4& v, uint64_t& key) {
    const int64_t p = p0 + lane / 8;
    if (p < c.end) v = reinterpret_cast<const uint4*>(&c.pods[p])[lane % 8];
    // port_off (bytes 92..95) sits in part 5's .w, port_cnt (96..99) in part 6's .x
    const int s = lane / PPK, k = lane % PPK;
    const int32_t off = __shfl((int32_t)v.w, s * 8 + 5, 64), cnt = __shfl((int32_t)v.x, s * 8 + 6, 64);
    key = 0;
    if (lane < RING_FILL * PPK && p0 + s < c.end && k < cnt && cnt <= PPK) key = c.pod_ports[off + k];
  };
  auto ring_store = [&](int64_t p0, const uint4& v, uint64_t key) {
    const int64_t p = p0 + lane / 8;
    if (p < c.end) reinterpret_cast<uint4*>(&s_pod[p % RING])[lane % 8] = v;
    if (lane < RING_FILL * PPK && p0 + lane / PPK < c.end) s_ppk[(p0 + lane / PPK) % RING][lane % PPK] = key;
  };
  if (wv == 1) {
    uint4 v = make_uint4(0, 0, 0, 0);
    uint64_t key;
    ring_load(c.first, v, key);
    ring_store(c.first, v, key);
  }
  if (tid == 0) {
    s_arr[0] = s_arr[1] = 0;
    s_done[0] = s_done[1] = -1;
    s_dec = 0;
    s_abort = 0;
    s_ev2[0] = s_ev2[1] = 0;
    s_mok[0] = s_mok[1] = 1;
    for (int w = 1; w < NW; ++w) {  // idle waves' partials: empty, for the combine and the masks
      if (active(w)) continue;
      for (int b = 0; b < 2; ++b) {
        s_fit[b][w] = 0;
        for (int q = 0; q < KSIM_MAX_RCLASS; ++q) {
          s_mx[b][w][q] = -1; s_cnt[b][w][q] = 0; s_mx2[b][w][q] = -1; s_cnt2[b][w][q] = 0; s_msk[b][w][q] = 0;
        }
      }
    }
  }
  uint64_t counter = *c.counter;  // replicated genericScheduler.lastNodeIndex (control wave)
  __syncthreads();

  auto pod_K = [&](const ksim_pod& P) -> int { return P.reserved[0] * P.reserved[1]; };
  // One row against pod V (the pod at ring slot p) → packed entry (ev_pack, -1 = does not fit)
  // and reason mask: ksim_predicates_a's predicatesOrdering chain (predicates.go:129-138)
  // evaluated branch-free on the LDS row, the map score in ksim_fast.h's float64 form
  // (bit-identical), the reduce class from the staged class tables.  d: the previous pod
  // committed to the row (dual hypothesis), or zero.
  auto eval_row = [&](const PodView& V, int64_t p, int32_t j, const RowDelta& d, uint32_t& rm) -> int32_t {
    // rare-path columns and tables through a laundered context pointer: loaded (scalar cache)
    // where a branch needs them instead of held in scalar registers across the pod loop
    const KsimCtx* cx = cg;
    asm volatile("" : "+s"(cx));
    KsimFastRow r;
    r.ac = RW[j].ac; r.am = RW[j].am; r.rc = RW[j].rc + d.c; r.rm = RW[j].rm + d.m; r.zc = RW[j].zc + d.zc;
    r.zm = RW[j].zm + d.zm; r.dac = RW[j].dac; r.dam = RW[j].dam;
    r.allowed = RW[j].allowed; r.count = RW[j].count + d.n; r.fl = RW[j].fl;
    if (d.g | d.e) {  // the previous pod's gpu / ephemeral request re-derives the over-commit bits
      const int64_t i = lo + j;
      r.fl &= ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
      if (cx->alloc_gpu[i] < cx->req_gpu[i] + d.g) r.fl |= KSIM_N_GPU_OVER;
      if (cx->alloc_eph[i] < cx->req_eph[i] + d.e) r.fl |= KSIM_N_EPH_OVER;
    }
    if (V.fast) {
      const KsimFastPod F{V.rq_c, V.rq_m, V.nz_c, V.nz_m, V.flags};
      return ksim_fast_eval(preds, F, r, no_prio, wl, wmr, wb, rm);
    }
    const int64_t i = lo + j;
    const int32_t ls = RW[j].ls, ts = RW[j].ts;
    const uint32_t fl = r.fl;
    // PodFitsResources (predicates.go:706-778)
    uint32_t res = (r.count + 1 > r.allowed) ? (1u << KSIM_R_INSUFFICIENT_PODS) : 0u;
    if (V.flags & KSIM_POD_ANY_REQUEST) {
      res |= (r.ac < V.rq_c + r.rc) ? (1u << KSIM_R_INSUFFICIENT_CPU) : 0u;
      res |= (r.am < V.rq_m + r.rm) ? (1u << KSIM_R_INSUFFICIENT_MEMORY) : 0u;
      if (V.rq_g == 0) res |= (fl & KSIM_N_GPU_OVER) ? (1u << KSIM_R_INSUFFICIENT_GPU) : 0u;
      else if (cx->alloc_gpu[i] < V.rq_g + cx->req_gpu[i] + d.g) res |= 1u << KSIM_R_INSUFFICIENT_GPU;
      if (V.rq_e == 0) res |= (fl & KSIM_N_EPH_OVER) ? (1u << KSIM_R_INSUFFICIENT_EPHEMERAL) : 0u;
      else if (cx->alloc_eph[i] < V.rq_e + cx->req_eph[i] + d.e) res |= 1u << KSIM_R_INSUFFICIENT_EPHEMERAL;
      for (int32_t s = 0; s < V.scalar_cnt; ++s) {
        const ksim_scalar_req q = cx->pod_scalars[V.scalar_off + s];
        const int64_t off = (int64_t)q.col * cx->n + i;
        if (cx->alloc_scalar[off] < q.req + cx->req_scalar[off]) res |= 1u << (KSIM_R_INSUFFICIENT_SCALAR0 + q.col);
      }
    }
    const uint32_t host = (V.host == -1 || V.host == i) ? 0u : (1u << KSIM_R_HOSTNAME);
    // PodFitsHostPorts (predicates.go:1019-1039, HostPortInfo.CheckConflict utils.go:101-130)
    uint32_t ports = 0;
    if (V.port_cnt) {
      const bool lk = V.port_cnt <= PPK;
      int32_t pc;
      if (L.ps) pc = reinterpret_cast<const int32_t*>(ksim_smem + L.off_pc)[j];
      else pc = cx->port_count[i];
      for (int32_t k = 0; k < V.port_cnt && !ports; ++k) {
        uint64_t want;
        if (lk) want = s_ppk[p % RING][k];
        else want = cx->pod_ports[V.port_off + k];
        const uint32_t wip = (uint32_t)(want >> 40);
        const uint64_t wpp = want & 0xFFFFFFFFFFull;
        bool hit = d.pp != 0;
        for (int32_t sl = 0; sl < pc && !hit; ++sl) {
          uint64_t e;
          if (L.ps) e = reinterpret_cast<const uint64_t*>(ksim_smem + L.off_pk)[sl * chunk + j];
          else e = cx->ports[(int64_t)sl * cx->n + i];
          if ((e & 0xFFFFFFFFFFull) != wpp) continue;
          const uint32_t eip = (uint32_t)(e >> 40);
          hit = wip == 0 || eip == 0 || eip == wip;
        }
        if (hit) ports = 1u << KSIM_R_HOST_PORTS;
      }
    }
    // podMatchesNodeLabels / tolerations: bits of the staged class tables
    uint32_t sel = 0, taint = 0, noexec = 0;
    uint32_t sv = 0;  // the (class, row) static bits when staged
    if (L.off_st) {
      sv = reinterpret_cast<const uint16_t*>(ksim_smem + L.off_st)[V.cls * chunk + j];
      if (V.flags & KSIM_POD_NEED_SELECTOR) sel = (sv & 1u) << KSIM_R_NODE_SELECTOR;
      if (V.flags & KSIM_POD_NEED_TAINTS) {
        taint = ((sv >> 1) & 1u) << KSIM_R_TAINTS;
        noexec = ((sv >> 2) & 1u) << KSIM_R_TAINTS;
      }
    } else if (V.flags & KSIM_POD_NEED_SELECTOR) {
      const int64_t w = (int64_t)V.cls * cx->lwords + (ls >> 5);
      uint32_t word;
      if (L.tables) word = reinterpret_cast<const uint32_t*>(ksim_smem + L.off_sel)[w];
      else word = cx->sel_ok[w];
      sel = ((word >> (ls & 31)) & 1u) ? 0u : (1u << KSIM_R_NODE_SELECTOR);
    }
    if (!L.off_st && (V.flags & KSIM_POD_NEED_TAINTS)) {
      const int64_t w = (int64_t)V.cls * cx->twords + (ts >> 5);
      uint32_t wt, wn;
      if (L.tables) {
        wt = reinterpret_cast<const uint32_t*>(ksim_smem + L.off_tok)[w];
        wn = reinterpret_cast<const uint32_t*>(ksim_smem + L.off_nok)[w];
      } else {
        wt = cx->taint_ok[w];
        wn = cx->noexec_ok[w];
      }
      taint = ((wt >> (ts & 31)) & 1u) ? 0u : (1u << KSIM_R_TAINTS);
      noexec = ((wn >> (ts & 31)) & 1u) ? 0u : (1u << KSIM_R_TAINTS);
    }
    // the first failing predicate in order (ksim_predicates_a)
    // Predicate enables as 32-bit integer masks (uniform, one scalar register each), node
    // conditions as per-lane bit moves: boolean selects on uniform conditions become 64-bit lane
    // masks the compiler hoists out of the pod loop and then spills
    // preds through a VGPR: a uniform condition would come back as a hoisted 64-bit lane mask
    uint32_t pr = preds;
    asm volatile("" : "+v"(pr));
    auto en = [&](uint32_t f) -> uint32_t { return 0u - ((pr / f) & 1u); };
    auto on = [](uint32_t v, uint32_t f, int r) -> uint32_t { return (uint32_t)((v & f) != 0u) << r; };
    uint32_t vf = V.flags;
    asm volatile("" : "+v"(vf));
    const uint32_t be = 0u - ((vf / KSIM_POD_BEST_EFFORT) & 1u);
    const uint32_t m_cond = en(KSIM_P_CHECK_NODE_CONDITION) & (fl & KSIM_COND_REASON_MASK);
    const uint32_t m_uns = en(KSIM_P_CHECK_NODE_UNSCHEDULABLE) & on(fl, KSIM_N_UNSCHEDULABLE, KSIM_R_UNSCHEDULABLE);
    const uint32_t m_gen = en(KSIM_P_GENERAL) & (res | host | ports | sel);
    const uint32_t m_host = en(KSIM_P_HOSTNAME) & host;
    const uint32_t m_ports = en(KSIM_P_HOST_PORTS) & ports;
    const uint32_t m_sel = en(KSIM_P_NODE_SELECTOR) & sel;
    const uint32_t m_res = en(KSIM_P_RESOURCES) & res;
    const uint32_t m_t = en(KSIM_P_TAINTS) & taint;
    const uint32_t m_nt = en(KSIM_P_NOEXEC_TAINTS) & noexec;
    const uint32_t m_lp = en(KSIM_P_LABEL_PRESENCE) & on(fl, KSIM_N_LABEL_PRESENCE, KSIM_R_LABEL_PRESENCE);
    const uint32_t m_mp = en(KSIM_P_MEM_PRESSURE) & be & on(fl, KSIM_N_MEM_PRESSURE, KSIM_R_MEM_PRESSURE);
    const uint32_t m_dp = en(KSIM_P_DISK_PRESSURE) & on(fl, KSIM_N_DISK_PRESSURE, KSIM_R_DISK_PRESSURE);
    uint32_t m = m_cond;
    for (const uint32_t x : {m_uns, m_gen, m_host, m_ports, m_sel, m_res, m_t, m_nt, m_lp, m_mp, m_dp}) m = m ? m : x;
    rm = m;
    if (m) return -1;
    const int32_t sc = no_prio ? 0 : (int32_t)ksim_fast_score(V.nz_c + r.zc, r.ac, r.dac, V.nz_m + r.zm, r.am, r.dam, wl, wmr, wb);
    int32_t cl = 0;
    if (V.k1 * V.k2 > 1) {
      int a = 0, b = 0;
      if (L.off_st) {
        a = V.k1 > 1 ? (int)((sv >> 4) & 15u) : 0;
        b = V.k2 > 1 ? (int)((sv >> 8) & 15u) : 0;
      } else if (V.k1 > 1) {
        const int64_t x = (int64_t)V.cls * cx->n_taint_sets + ts;
        if (L.tables) a = (uint8_t)(ksim_smem + L.off_ttc)[x];
        else a = cx->tt_class[x];
      }
      if (!L.off_st && V.k2 > 1) {
        const int64_t x = (int64_t)V.cls * cx->n_label_sets + ls;
        if (L.tables) b = (uint8_t)(ksim_smem + L.off_nac)[x];
        else b = cx->na_class[x];
      }
      cl = a * V.k2 + b;
    }
    return ev_pack(true, cl, sc);
  };
  // The delta pod `p` makes to a row when committed, if the dual hypothesis can express it: not
  // when both pods carry scalar resources, nor beyond PPK host ports (host ports go through the
  // pair-conflict flag against pod q; gpu / ephemeral through re-derived over-commit bits).
  auto delta_of = [&](int64_t p, int64_t q, RowDelta& d) -> bool {
    const ksim_pod& P = s_pod[p % RING];
    const ksim_pod& Q = s_pod[q % RING];
    if (P.scalar_cnt && Q.scalar_cnt) return false;
    if (P.port_cnt > PPK || Q.port_cnt > PPK) return false;
    d.c = P.add_cpu; d.m = P.add_mem; d.zc = P.nz_cpu; d.zm = P.nz_mem; d.n = 1; d.pp = 0;
    d.g = P.add_gpu; d.e = P.add_eph;
    // HostPortInfo.CheckConflict of Q's wanted keys against P's (utils.go:101-130)
    for (int32_t a = 0; a < Q.port_cnt; ++a) {
      const uint64_t want = s_ppk[q % RING][a];
      const uint32_t wip = (uint32_t)(want >> 40);
      for (int32_t b = 0; b < P.port_cnt; ++b) {
        const uint64_t e = s_ppk[p % RING][b];
        if ((e & 0xFFFFFFFFFFull) != (want & 0xFFFFFFFFFFull)) continue;
        const uint32_t eip = (uint32_t)(e >> 40);
        if (wip == 0 || eip == 0 || eip == wip) d.pp = 1;
      }
    }
    return true;
  };
  // row wave: pod p's entries (ev) for this lane's rows → LDS ev / rm1; with `hyp`, also the
  // entries with pod p-1 committed to each row (ev2 / rm2) — on the next waves up when the rows
  // fit one wave set each (split), else after ev on the same lane.  One evaluation call site,
  // so one inlined copy; the partial reads the entries back from LDS.
  auto eval_rows = [&](const PodView& V, int64_t p, bool hyp, const RowDelta& d, int32_t (&e)[NPT], int buf) {
#ifdef KSIM_STAMPS
    const uint64_t q0 = __builtin_amdgcn_s_memtime();
    const uint64_t q1 = q0;
#endif
    const RowDelta z{0, 0, 0, 0, 0, 0, 0, 0};
    const int32_t half = split ? 64 * ((nrows + 63) / 64) : 0;  // split: ev2 threads start here
    const int ntask = split ? 1 : NPT * (hyp ? 2 : 1);
#pragma unroll 1
    for (int t = 0; t < ntask; ++t) {
      int32_t j;
      bool h;
      if (split) {
        h = rt >= half;
        j = h ? rt - half : rt;
        if (h && !hyp) j = nrows;  // nothing to do
      } else {
        h = hyp && (t & 1);
        j = (hyp ? t >> 1 : t) * RT + rt;
      }
      if (j < nrows) {
        uint32_t m;
        const int32_t x = eval_row(V, p, j, h ? d : z, m);
        if (h) { RW[j].ev2[buf] = x; RW[j].rm2[buf] = m; }
        else { RW[j].ev[buf] = x; RW[j].rm1[buf] = m; }
      }
    }
#ifdef KSIM_STAMPS
    const uint64_t q2 = __builtin_amdgcn_s_memtime();
#endif
    // this lane's entries for the partial (split: the ev threads' only)
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int k = 0; k < NPT; ++k) {
      const int32_t j = k * RT + rt;
      e[k] = (j < nrows && !(split && rt >= half)) ? RW[j].ev[buf] : -1;
    }
#ifdef KSIM_STAMPS
    const uint64_t q3 = __builtin_amdgcn_s_memtime();
    ev_acc[0] += q1 - q0; ev_acc[1] += q2 - q1; ev_acc[2] += q3 - q2; ev_acc[3] += 1;
#endif
  };
  // (fit count, per class: top value / count, second value / count) of one row wave → LDS slot w.
  // Four classes at a time: their DPP reductions are independent chains that interleave.
  auto partial = [&](const int32_t (&e)[NPT], int K, int buf, int w) {
    int32_t nf = 0;
#pragma unroll
    for (int k = 0; k < NPT; ++k) nf += __popcll(__ballot(e[k] >= 0));
    if (lane == 0) s_fit[buf][w] = nf;
    // U classes per group (their DPP chains are independent and interleave); the group width
    // follows K so a one- or two-class pod runs one or two chains, not four
    auto group = [&](int q0, auto UU) {
      constexpr int U = decltype(UU)::value;
      int32_t v[U], wm[U], n[U], v2[U], wm2[U], n2[U];
      uint64_t mk[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        v[u] = -1;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const bool in = e[k] >= 0 && (K == 1 || ev_cls(e[k]) == q0 + u);
          const int32_t sc = K == 1 ? e[k] : ev_score(e[k]);
          v[u] = (in && sc > v[u]) ? sc : v[u];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) wm[u] = ksimw::max_i32(v[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        n[u] = 0;
        v2[u] = -1;
        mk[u] = 0;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const bool in = e[k] >= 0 && (K == 1 || ev_cls(e[k]) == q0 + u);
          const int32_t sc = K == 1 ? e[k] : ev_score(e[k]);
          const uint64_t b = __ballot(in && sc == wm[u]);
          mk[u] = b;
          n[u] += __popcll(b);
          v2[u] = (in && sc < wm[u] && sc > v2[u]) ? sc : v2[u];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) wm2[u] = ksimw::max_i32(v2[u]);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        n2[u] = 0;
#pragma unroll
        for (int k = 0; k < NPT; ++k) {
          const bool in = e[k] >= 0 && (K == 1 || ev_cls(e[k]) == q0 + u);
          const int32_t sc = K == 1 ? e[k] : ev_score(e[k]);
          n2[u] += __popcll(__ballot(in && wm2[u] >= 0 && sc == wm2[u]));
        }
      }
      if (lane == 0) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          if (q0 + u >= K) break;
          s_mx[buf][w][q0 + u] = wm[u]; s_cnt[buf][w][q0 + u] = wm[u] < 0 ? 0 : n[u];
          s_mx2[buf][w][q0 + u] = wm2[u]; s_cnt2[buf][w][q0 + u] = wm2[u] < 0 ? 0 : n2[u];
          if (NPT == 1) s_msk[buf][w][q0 + u] = wm[u] < 0 ? 0ull : mk[u];
        }
      }
    };
    if (K == 1) group(0, std::integral_constant<int, 1>{});
    else if (K == 2) group(0, std::integral_constant<int, 2>{});
    else
      for (int q0 = 0; q0 < K; q0 += 4) group(q0, std::integral_constant<int, 4>{});
  };
  // the last row wave of a pod: combine the row waves' partials (lane q = class q) into the
  // workgroup's top two per class → LDS (the owner's correction) and the granule payloads
  auto combine = [&](int K, int buf) -> uint64_t {
    const int q = lane < K ? lane : 0;
    int32_t f = 0, mx[NW], cn[NW], mx2[NW], cn2[NW];
#pragma unroll
    for (int w = 1; w < NW; ++w) {  // all loads first: one LDS round trip
      f += s_fit[buf][w];
      mx[w] = s_mx[buf][w][q];
      cn[w] = s_cnt[buf][w][q];
      mx2[w] = s_mx2[buf][w][q];
      cn2[w] = s_cnt2[buf][w][q];
    }
    int32_t m = -1, n = 0;
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const bool up = cn[w] != 0 && mx[w] > m, eq = cn[w] != 0 && mx[w] == m;
      n = up ? cn[w] : (eq ? n + cn[w] : n);
      m = up ? mx[w] : m;
    }
    // second value: the best below m among the waves' tops and seconds
    int32_t m2 = -1, n2 = 0;
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      const int32_t a = (cn[w] != 0 && mx[w] < m) ? mx[w] : (cn2[w] != 0 ? mx2[w] : -1);
      m2 = a > m2 ? a : m2;
    }
#pragma unroll
    for (int w = 1; w < NW; ++w) {
      if (m2 < 0) break;
      n2 += (cn[w] != 0 && mx[w] == m2) ? cn[w] : 0;
      n2 += (cn2[w] != 0 && mx2[w] == m2) ? cn2[w] : 0;
    }
    if (lane < K) s_top[buf][lane] = make_int4(m, n, m2, n2);
    if (lane == 0) s_F[buf] = f;
    if (lane >= K) return 0;
    return (lane == 0 ? ((uint64_t)f << 44) : 0) | ((uint64_t)n << 32) | (uint64_t)(uint32_t)m;
  };
  auto ptag = [&](int64_t p) -> uint64_t { return (uint64_t)((p - c.first + 1) & 0xFF); };
  // row waves: the last one to finish pod p's partial combines and publishes it
  auto arrive_publish = [&](int64_t p, int K, int buf) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    // per-parity counter: a row wave can run a pod ahead of its slower siblings (the waves are
    // decoupled), never two, so pods of one parity never mix; the last arriver re-arms it
    int32_t old = 0;
    if (lane == 0) old = atomicAdd(&s_arr[buf], 1);
    old = __builtin_amdgcn_readfirstlane(old);
    if (old + 1 == nact) {
      PROBE(10);
      if (lane == 0) s_arr[buf] = 0;
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
      const uint64_t v = combine(K, buf);
      if (lane < K) store_granule(spec_at<MB>(granules, (int)(p % NSLOT), blockIdx.x, lane), (ptag(p) << 56) | v);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&s_done[buf], (int32_t)ptag(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
  };

  // ---- prologue: partial of the first pod ----
  if (wv > 0 && active(wv)) {
    int32_t e[NPT];
    const int K0 = pod_K(s_pod[c.first % RING]);
    const RowDelta z{0, 0, 0, 0, 0, 0, 0, 0};
    eval_rows(pod_view_lds(&s_pod[c.first % RING]), c.first, false, z, e, (int)(c.first & 1));
    partial(e, K0, c.first & 1, wv);
    arrive_publish(c.first, K0, c.first & 1);
  }
  int X = -1;  // control wave: owner workgroup of the previous pod's node (-1: none)
  __syncthreads();
#ifdef KSIM_STAMPS
  uint64_t t_prev = __builtin_amdgcn_s_memtime();
#endif

  // The two roles run decoupled, synchronised through LDS only: the row waves evaluate pod + 1
  // once the control wave has committed every pod up to pod - 1 (s_dec), the control wave's
  // owner correction waits for the row waves' pod + 1 statistics (s_done).
  if (wv == 0) {
  for (int64_t pod = c.first; pod < c.end; ++pod) {
    const bool has_next = pod + 1 < c.end;
    const int pb = (int)(pod & 1);        // LDS buffers of pod
    const int nb = (int)((pod + 1) & 1);  // LDS buffers of pod + 1
#ifdef KSIM_STAMPS
    uint64_t o_prev = 0;
#endif

      const ksim_pod& P = s_pod[pod % RING];
      const int K = pod_K(P);
      const int k2 = P.reserved[1];
      // the reduce classes' map values (lane q = class q), loaded now, used after the sweep
      int64_t tv_l = 0, av_l = 0, ad_l = 0;
      if (K > 1 && lane < K) {
        const int64_t* ttv = L.tables ? reinterpret_cast<const int64_t*>(ksim_smem + L.off_ttv) : c.tt_val;
        const int64_t* nav = L.tables ? reinterpret_cast<const int64_t*>(ksim_smem + L.off_nav) : c.na_val;
        tv_l = ttv[(int64_t)P.cls * c.val_w + lane / k2];
        av_l = nav[(int64_t)P.cls * c.val_w + lane % k2];
        if (c.na_add) {
          const int64_t* nad = L.tables ? reinterpret_cast<const int64_t*>(ksim_smem + L.off_nad) : c.na_add;
          ad_l = nad[(int64_t)P.cls * c.val_w + lane % k2];
        }
      }
      // ---------------- a. sweep: every speculative partial of pod + the owner's correction ----
      const uint64_t tag = ptag(pod);
      const int slot = (int)(pod % NSLOT);
      STAMP(1);
      uint64_t g[MB];
      uint64_t gq[KF][MB];  // granules of classes 1..KF, kept in registers (LDS beyond)
      bool ok = false;
      const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#ifdef KSIM_STAMPS
      bool seen_spec = false, seen_fix = false;
#endif
      for (;;) {
        // unconditional loads (slots are sized for MAXG workgroups): one fabric round trip for
        // class 0, the owner's correction and (KF at a time) the further reduce classes
#pragma unroll
        for (int j = 0; j < MB; ++j) g[j] = load_granule(spec_at<MB>(granules, slot, lane * MB + j, 0));
        const uint64_t fx = load_granule(fix_at(granules, slot, 0));
        bool mine = X < 0 || gtag(fx) == tag;
#pragma unroll
        for (int j = 0; j < MB; ++j) {
          const int b = lane * MB + j;
          mine &= (b >= G) || b == X || gtag(g[j]) == tag;
        }
        for (int q0 = 1; q0 < K; q0 += KF) {  // classes >= 1 were published with class 0
          uint64_t v[KF][MB];
#pragma unroll
          for (int u = 0; u < KF; ++u)
#pragma unroll
            for (int j = 0; j < MB; ++j) {
              const int b = lane * MB + j;
              v[u][j] = (q0 + u < K && b < G) ? load_granule(gran_at<MB>(granules, slot, b, q0 + u, X)) : 0;
            }
#pragma unroll
          for (int u = 0; u < KF; ++u)
#pragma unroll
            for (int j = 0; j < MB; ++j) {
              const int b = lane * MB + j;
              if (q0 + u < K && b < G) mine &= gtag(v[u][j]) == tag;
              if (q0 == 1) gq[u][j] = v[u][j];
              else if (q0 + u < K && b < G) s_gq[q0 + u - 1 - KF][b] = v[u][j];
            }
        }
#ifdef KSIM_STAMPS
        st_acc[8] += 1;
        {
          bool sp = true;
#pragma unroll
          for (int j = 0; j < MB; ++j) sp &= (lane * MB + j >= G) || lane * MB + j == X || gtag(g[j]) == tag;
          const uint64_t tn = __builtin_amdgcn_s_memtime();
          if (!seen_spec && __all(sp)) { seen_spec = true; st_acc[12] += tn - t_prev; }
          if (!seen_fix && (X < 0 || gtag(fx) == tag)) { seen_fix = true; st_acc[13] += tn - t_prev; }
        }
#endif
        if (__all(mine)) {
          ok = true;
#pragma unroll
          for (int j = 0; j < MB; ++j) g[j] = (lane * MB + j == X) ? fx : g[j];
          break;
        }
        if (__builtin_amdgcn_s_memrealtime() - t0 > SPIN_LIMIT_TICKS) break;
        __builtin_amdgcn_s_sleep(1);
      }
      STAMP(2);
      PROBE(2);
#pragma unroll
      for (int j = 0; j < MB; ++j) g[j] = (lane * MB + j < G) ? g[j] : 0;
      ok = __all(ok);
      int32_t F = 0, M0 = -1, C0 = 0;
      if (ok) {
        int32_t f = 0, m = -1, n = 0;
#pragma unroll
        for (int j = 0; j < MB; ++j) {
          f += gfit(g[j]);
          const int32_t cnt = gcnt(g[j]), s = gscore(g[j]);
          if (cnt == 0) continue;
          if (s > m) { m = s; n = cnt; }
          else if (s == m) n += cnt;
        }
        F = ksimw::sum_i32(f);
        M0 = ksimw::max_i32(n ? m : -1);
        C0 = ksimw::sum_i32((n && m == M0) ? n : 0);
      }
      STAMP(9);
      // lane q: reduce class q's global maximum and its count (registers: the control wave's
      // LDS round trips queue behind the row waves' evaluation traffic)
      int32_t mq_l = lane == 0 ? M0 : -1, cq_l = lane == 0 ? C0 : 0;
      if (ok && K > 1) {  // further reduce classes (TaintToleration x NodeAffinity), swept above
        auto class_stat = [&](int q, const uint64_t (&v)[MB]) {
          int32_t mm = -1, nn = 0;
#pragma unroll
          for (int j = 0; j < MB; ++j) {
            const int b = lane * MB + j;
            const int32_t cnt = b < G ? gcnt(v[j]) : 0, s = gscore(v[j]);
            if (cnt == 0) continue;
            if (s > mm) { mm = s; nn = cnt; }
            else if (s == mm) nn += cnt;
          }
          const int32_t Mq = ksimw::max_i32(nn ? mm : -1);
          const int32_t Cq = ksimw::sum_i32((nn && mm == Mq) ? nn : 0);
          mq_l = lane == q ? Mq : mq_l;
          cq_l = lane == q ? Cq : cq_l;
        };
#pragma unroll
        for (int u = 0; u < KF; ++u)
          if (1 + u < K) class_stat(1 + u, gq[u]);
        for (int q = 1 + KF; q < K; ++q) {
          uint64_t v[MB];
#pragma unroll
          for (int j = 0; j < MB; ++j) v[j] = lane * MB + j < G ? s_gq[q - 1 - KF][lane * MB + j] : 0;
          class_stat(q, v);
        }
      }
      STAMP(11);
      int mode = 0, blk = -1, rank = 0;
      uint32_t win = 1;
      int32_t tgt = -2;  // lane q: the packed entry a winning row of class q has (select), -2 none
      if (!ok) {
        mode = -1;
        if (lane == 0) atomicOr(c.err, 4);
      } else if (F > 0) {
        mode = 1;
        int64_t ix = 0;
        if (F > 1) {  // generic_scheduler.go:153-156: a single fit skips selectHost
          mode = 2;
          int64_t C = C0;
          if (K > 1) {
            // lane q = reduce class q, all at once: NormalizeReduce's maxima over the filtered
            // set (classes with fit nodes), each class's weighted total, the best total and the
            // classes that reach it (reduce.go:29-64, generic_scheduler.go:632-639)
            const bool live = lane < K && cq_l != 0;
            const int32_t cq = live ? cq_l : 0;
            const int64_t mq = live ? mq_l : 0;
            const int64_t mxT = wave_max_i64(live ? tv_l : 0), mxA = wave_max_i64(live ? av_l : 0);
            const int64_t t = live ? class_total(c, tv_l, av_l, ad_l, mq, mxT, mxA) : -1;  // totals are >= 0
            const int64_t best = wave_max_i64(t);
            const uint64_t wbm = __ballot(live && t == best);
            win = (uint32_t)wbm;
            C = ksimw::sum_i32((wbm >> lane) & 1ull ? cq : 0);
            tgt = ((wbm >> lane) & 1ull) ? ((lane << EV_SHIFT) | (int32_t)mq) : -2;
          } else {
            tgt = lane == 0 ? M0 : -2;
          }
          ix = (counter >> 32) ? (int64_t)(counter % (uint64_t)C) : (int64_t)((uint32_t)counter % (uint32_t)C);
          counter += 1;  // generic_scheduler.go:192-195
        }
        STAMP(10);
        // ---- locate the workgroup holding the ix-th match counted from the top ----
        int32_t bm[MB];
        int32_t tot = 0;
#pragma unroll
        for (int j = 0; j < MB; ++j) {
          const int b = lane * MB + j;
          int32_t m = 0;
          if (b < G) {
            if (mode == 1) {
              m = gfit(g[j]);
            } else {
              if ((win & 1u) && gcnt(g[j]) && gscore(g[j]) == M0) m += gcnt(g[j]);
#pragma unroll
              for (int u = 0; u < KF; ++u) {
                const int q = 1 + u;
                if (q >= K || !((win >> q) & 1u)) continue;
                const uint64_t v = gq[u][j];
                if (gcnt(v) && gscore(v) == __builtin_amdgcn_readlane(mq_l, q)) m += gcnt(v);
              }
              for (int q = 1 + KF; q < K; ++q) {
                if (!((win >> q) & 1u)) continue;
                const uint64_t v = s_gq[q - 1 - KF][b];
                if (gcnt(v) && gscore(v) == __builtin_amdgcn_readlane(mq_l, q)) m += gcnt(v);
              }
            }
          }
          bm[j] = m;
          tot += m;
        }
        const int32_t pre = ksimw::prefix_incl_i32(tot);
        const int32_t total = __builtin_amdgcn_readlane(pre, 63);
        const int64_t above = (int64_t)(total - pre);  // matches in workgroups of higher lanes
        const bool hit = tot > 0 && ix >= above && ix < above + tot;
        int32_t found = -1, r = 0;
        if (hit) {
          int64_t rr = ix - above;
#pragma unroll
          for (int j = MB - 1; j >= 0; --j) {
            if (found < 0) {
              if (rr < bm[j]) found = lane * MB + j;
              else rr -= bm[j];
            }
          }
          r = (int32_t)rr;
        }
        const uint64_t hb = __ballot(hit);
        if (hb == 0) {
          mode = -1;
        } else {
          const int src = __builtin_ffsll((long long)hb) - 1;
          blk = __builtin_amdgcn_readlane(found, src);
          rank = __builtin_amdgcn_readlane(r, src);
          if (blk < 0) mode = -1;
        }
        if (mode < 0 && lane == 0) atomicOr(c.err, 2);
      }
      STAMP(3);
#ifdef KSIM_STAMPS
      o_prev = __builtin_amdgcn_s_memtime();
#endif
      if (mode > 0 && blk == (int)blockIdx.x) {
        // ---------------- d. owner: exact row (rank from the top), correction, commit ----------
        int32_t jsel = -1;
        if (NPT == 1 && mode == 2 && s_mok[pb]) {
          // from the row waves' top masks: lane w = row wave w's rows at a winning class's
          // maximum (a wave whose top is below the class maximum holds none of them)
          uint64_t cm = 0;
          for (uint32_t wq = win; wq; wq &= wq - 1) {
            const int q = __builtin_ctz(wq);
            const int32_t t = __builtin_amdgcn_readlane(tgt, q);
            const int32_t ts = K == 1 ? t : ev_score(t);
            if (lane >= 1 && lane < NW && s_cnt[pb][lane][q] && s_mx[pb][lane][q] == ts) cm |= s_msk[pb][lane][q];
          }
          int32_t rr = rank;
#pragma unroll
          for (int w = NW - 1; w >= 1; --w) {  // rows of wave w: (w-1)*64 + lane; the top first
            if (jsel >= 0) break;
            const uint64_t m = (uint64_t)readlane64((int64_t)cm, w);
            const int nbits = __popcll(m);
            if (rr >= nbits) { rr -= nbits; continue; }
            const bool is = ((m >> lane) & 1ull) && __popcll((m >> lane) >> 1) == rr;
            jsel = (w - 1) * 64 + (__builtin_ffsll((long long)__ballot(is)) - 1);
          }
        }
        if (jsel < 0) {
          // scan pod's entries from the top: 64-row segments, four per LDS round trip
          int32_t rr = rank;
          const int nseg = (nrows + 63) / 64;
          for (int s0 = nseg - 1; s0 >= 0 && jsel < 0; s0 -= 4) {
            uint64_t bl[4];
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              const int32_t j = (s0 - u) * 64 + lane;
              const int32_t e = (s0 - u >= 0 && j < nrows) ? RW[j].ev[pb] : -1;
              bool mt = e >= 0;
              if (mode == 2) {  // one compare per winning class (usually one)
                mt = false;
                for (uint32_t wq = win; wq; wq &= wq - 1)
                  mt |= e == __builtin_amdgcn_readlane(tgt, __builtin_ctz(wq));
              }
              bl[u] = __ballot(mt);
            }
#pragma unroll
            for (int u = 0; u < 4; ++u) {
              if (jsel >= 0) break;
              uint64_t m = bl[u];
              const int nbits = __popcll(m);
              if (rr >= nbits) { rr -= nbits; continue; }
              // the rr-th set bit from the top: set, with exactly rr set bits above it
              const bool is = ((m >> lane) & 1ull) && __popcll((m >> lane) >> 1) == rr;
              const uint64_t bb = __ballot(is);
              jsel = (s0 - u) * 64 + (__builtin_ffsll((long long)bb) - 1);
            }
          }
        }
        OSTAMP(22);
        PROBE(3);
        if (jsel < 0) {
          mode = -1;
          if (lane == 0) atomicOr(c.err, 2);
        } else {
          const bool side = (P.add_gpu | P.add_eph | P.scalar_cnt | P.port_cnt) != 0;
          // NodeInfo.AddPod on the row: LDS columns, then the side columns (HBM / LDS ports).
          // Only after the row waves' pod + 1 evaluation is complete: they read this row.
          auto commit_row = [&]() {
            if (lane == 0) {
              RW[jsel].rc += P.add_cpu; RW[jsel].rm += P.add_mem; RW[jsel].zc += P.nz_cpu; RW[jsel].zm += P.nz_mem;
              RW[jsel].count += 1;
              if (side) {
                const bool lds_ports = P.port_cnt && L.ps;
                uint32_t fl = RW[jsel].fl;
                if (P.add_gpu | P.add_eph | P.scalar_cnt | (P.port_cnt && !L.ps)) {
                  fl = commit_side(cg, &P, lo + jsel, fl, lds_ports ? 0 : 1);
                  RW[jsel].fl = fl;
                }
                if (lds_ports) commit_ports_lds(cg, &P, lo + jsel, jsel, (int32_t)chunk, L.off_pc, L.off_pk);
              }
            }
          };
          // pods through `pod` committed: the row waves may evaluate pod + 2 (their chain to the
          // next-but-one decision starts here, so the owner releases them before its bookkeeping)
          auto release_dec = [&]() {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
            if (lane == 0) __hip_atomic_store(&s_dec, (int32_t)(pod - c.first + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
          };
          OSTAMP(23);
          if (has_next) {
            // the row waves' pod + 1 stats (and ev2) must be complete
            const int32_t want = (int32_t)ptag(pod + 1);
            while (__hip_atomic_load(&s_done[nb], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != want)
              __builtin_amdgcn_s_sleep(1);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
            const ksim_pod& Q = s_pod[(pod + 1) % RING];
            const int Kn = pod_K(Q);
            const int q = lane < Kn ? lane : 0;
            // one LDS round trip: the workgroup's top two, the row's two entries, the flags
            const int4 t = s_top[nb][q];
            const int32_t fN = s_F[nb];
            const int32_t e1 = RW[jsel].ev[nb];
            const bool dual = s_ev2[nb] != 0;
            const int32_t mok = s_mok[nb];
            int32_t e2 = RW[jsel].ev2[nb];
            uint32_t rm2 = RW[jsel].rm2[nb];
            if (!dual) {  // commit everything, then evaluate the one row here
              commit_row();
              release_dec();
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
              __builtin_amdgcn_wave_barrier();
              __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
              const RowDelta z{0, 0, 0, 0, 0, 0, 0, 0};
              e2 = eval_row(pod_view(Q), pod + 1, jsel, z, rm2);
            }
            OSTAMP(16);
            // O(1) correction of this workgroup's pod + 1 partial: e1 leaves its class, e2 joins
            // (the reduce class is the row's, the same for both when both fit)
            int32_t f = fN - (e1 >= 0) + (e2 >= 0);
            int32_t m = t.x, n = t.y;
            const int q1 = e1 < 0 ? -1 : (Kn == 1 ? 0 : ev_cls(e1));
            const int32_t s1 = Kn == 1 ? e1 : ev_score(e1);
            if (q1 == q && s1 == m) {
              if (n > 1) n -= 1;
              else { m = t.z; n = t.w; }
            }
            const int q2 = e2 < 0 ? -1 : (Kn == 1 ? 0 : ev_cls(e2));
            const int32_t s2 = Kn == 1 ? e2 : ev_score(e2);
            if (q2 == q) {
              if (n == 0 || s2 > m) { m = s2; n = 1; }
              else if (s2 == m) n += 1;
            }
            if (n == 0) m = -1;
            const uint64_t v = (lane == 0 ? ((uint64_t)f << 44) : 0) | ((uint64_t)n << 32) | (uint64_t)(uint32_t)m;
            if (lane < Kn) store_granule(fix_at(granules, (int)((pod + 1) % NSLOT), lane), (ptag(pod + 1) << 56) | v);
            OSTAMP(19);
            PROBE(4);
            if (dual) {
              commit_row();
              release_dec();
            }
            if (lane == 0) {
              RW[jsel].ev[nb] = e2;
              RW[jsel].rm1[nb] = rm2;
              // the same replacement in row wave wj's top masks (one row per row thread)
              if (NPT == 1 && mok) {
                const int wj = 1 + jsel / 64;
                const uint64_t bit = 1ull << (jsel % 64);
                bool keep = true;
                if (q1 >= 0 && s_cnt[nb][wj][q1] && s_mx[nb][wj][q1] == s1) {
                  s_msk[nb][wj][q1] &= ~bit;
                  const int32_t cn = s_cnt[nb][wj][q1] - 1;
                  s_cnt[nb][wj][q1] = cn;
                  keep = cn > 0;  // the wave's next value's rows are not recorded: scan
                }
                if (keep && q2 >= 0) {
                  const int32_t cn = s_cnt[nb][wj][q2], tv = s_mx[nb][wj][q2];
                  if (cn == 0 || s2 > tv) { s_mx[nb][wj][q2] = s2; s_cnt[nb][wj][q2] = 1; s_msk[nb][wj][q2] = bit; }
                  else if (s2 == tv) { s_cnt[nb][wj][q2] = cn + 1; s_msk[nb][wj][q2] |= bit; }
                }
                if (!keep) s_mok[nb] = 0;
              }
            }
#ifdef KSIM_STAMPS
            if (lane == 0) atomicAdd((unsigned long long*)&c.dbg[21], 1ull);
#endif
          } else {
            commit_row();
          }
          if (lane == 0) c.out_node[pod] = (int32_t)(lo + jsel);
          OSTAMP(20);
        }
      }
      if (mode == 0 && blockIdx.x == 0 && lane == 0) c.out_node[pod] = -1;
      X = mode > 0 ? blk : -1;
      STAMP(6);
      if (mode < 0) {  // uniform: every workgroup reaches the same verdict
        if (lane == 0) __hip_atomic_store(&s_abort, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
        break;
      }
      if (mode == 0 && c.collect && c.out_reasons) {  // FitError: every workgroup adds its rows' reasons
        int32_t acc = 0;
        for (int32_t j0 = 0; j0 < nrows; j0 += 64) {
          const int32_t j = j0 + lane;
          const uint32_t rm = j < nrows ? RW[j].rm1[pb] : 0u;
#pragma unroll
          for (int r = 0; r < KSIM_NREASONS; ++r) {
            const int32_t n = __popcll(__ballot((rm >> r) & 1u));
            acc += lane == r ? n : 0;
          }
        }
        if (lane < KSIM_NREASONS && acc) atomicAdd(&c.out_reasons[pod * KSIM_NREASONS + lane], acc);
      }
      // pods through `pod` are decided and committed: the row waves may evaluate pod + 2
      PROBE(5);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      if (lane == 0) __hip_atomic_store(&s_dec, (int32_t)(pod - c.first + 1), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      STAMP(4);
    }
  } else if (active(wv)) {
  for (int64_t pod = c.first; pod < c.end; ++pod) {
    const bool has_next = pod + 1 < c.end;
    const int nb = (int)((pod + 1) & 1);  // LDS buffers of pod + 1
#ifdef KSIM_STAMPS
    uint64_t o_prev = 0;
#endif

      // ---------------- b. speculative evaluation of pod + 1 (row waves) ----------------
      // wave 1 refills the descriptor ring every RING_FILL pods; the load's latency hides
      // under the evaluation (the control wave is at most one pod behind the row waves)
      const bool refill = wv == 1 && ((pod - c.first) % RING_FILL) == 0;
      uint4 rv = make_uint4(0, 0, 0, 0);
      uint64_t rkey = 0;
      if (refill) ring_load(pod + RING_FILL, rv, rkey);
#ifdef KSIM_STAMPS
      const uint64_t te0 = __builtin_amdgcn_s_memtime();
#endif
      if (has_next) {
        // pod + 1 is evaluated on the rows as committed through pod - 1 (the hypothesis covers pod).
        // The pod view and the commit delta need only the ring: before the wait, off the chain.
        PodView V = pod_view_lds(&s_pod[(pod + 1) % RING]);
        const int Kn = pod_K(s_pod[(pod + 1) % RING]);
        RowDelta d{0, 0, 0, 0, 0, 0, 0, 0};
        const bool hyp = delta_of(pod, pod + 1, d);
        const int32_t need = (int32_t)(pod - c.first);
#ifdef KSIM_STAMPS
        const uint64_t tw0 = __builtin_amdgcn_s_memtime();
#endif
        while (__hip_atomic_load(&s_dec, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) < need &&
               !__hip_atomic_load(&s_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP))
          __builtin_amdgcn_s_sleep(1);
#ifdef KSIM_STAMPS
        if (tid == 64) wait_acc += __builtin_amdgcn_s_memtime() - tw0;
#endif
        if (__hip_atomic_load(&s_abort, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) break;
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup");
        PROBE(1);
        PROBE_IF(7, wv == 1);
        PROBE_IF(8, wv == 3);
        PROBE_IF(9, wv >= 5);
        PROBE_IF(11, wv == 2);
        int32_t e[NPT];
        if (tid == 64) {
          s_ev2[nb] = hyp ? 1 : 0;
          s_mok[nb] = 1;
        }
        eval_rows(V, pod + 1, hyp, d, e, nb);
#ifdef KSIM_STAMPS
        const uint64_t te1 = __builtin_amdgcn_s_memtime();
        if (tid == 64) st_acc[14] += te1 - te0;
#endif
        partial(e, Kn, nb, wv);
#ifdef KSIM_STAMPS
        const uint64_t te2 = __builtin_amdgcn_s_memtime();
        if (tid == 64) st_acc[15] += te2 - te1;
#endif
        PROBE(6);
        arrive_publish(pod + 1, Kn, nb);
      }
#ifdef KSIM_STAMPS
      if (tid == 64) st_acc[5] += __builtin_amdgcn_s_memtime() - te0;
#endif
      if (refill) ring_store(pod + RING_FILL, rv, rkey);
    }
  }
  // the table is authoritative in HBM between calls: write the owned rows back
  __syncthreads();
  for (int32_t j = tid; j < nrows; j += BS) {
    const int64_t i = lo + j;
    c.req_cpu[i] = RW[j].rc; c.req_mem[i] = RW[j].rm;
    c.nz_cpu[i] = RW[j].zc; c.nz_mem[i] = RW[j].zm;
    c.pod_count[i] = RW[j].count; c.flags[i] = RW[j].fl;
  }
  if (blockIdx.x == 0 && tid == 0) {
    *c.counter = counter;
    *c.cursor = c.end;
  }
#ifdef KSIM_STAMPS
  if (blockIdx.x == 0 && tid == 0)
    for (int k = 0; k < 16; ++k) c.dbg[k] += (k == 5) ? 0 : st_acc[k];
  if (blockIdx.x == 0 && tid == 64) {
    c.dbg[5] += st_acc[5]; c.dbg[24] += st_acc[14]; c.dbg[25] += st_acc[15];
    for (int k = 0; k < 4; ++k) c.dbg[26 + k] += ev_acc[k];
    c.dbg[30] += wait_acc;
  }
#endif
}

// Checks the DPP wave helpers against plain lane loops (diagnostic, tests/ only).
__global__ void ksim_wave_selftest_kernel(int32_t* out) {
  const int lane = threadIdx.x;
  const int32_t v = (int32_t)((lane * 7919 + 13) % 97) - 40 + (blockIdx.x * 11);
  out[(blockIdx.x * 3 + 0) * 64 + lane] = ksimw::max_i32(v);
  out[(blockIdx.x * 3 + 1) * 64 + lane] = ksimw::sum_i32(v);
  out[(blockIdx.x * 3 + 2) * 64 + lane] = ksimw::prefix_incl_i32(v);
}

// ---------------------------------------------------------------------------------------
static constexpr int LDS_BUDGET = 120 * 1024;

static int num_cus() {
  int dev = 0;
  hipDeviceProp_t p;
  if (hipGetDevice(&dev) != hipSuccess || hipGetDeviceProperties(&p, dev) != hipSuccess) return 0;
  return p.multiProcessorCount;
}

// One workgroup per CU (<= 256) so every workgroup is resident — the protocol spins on every
// other workgroup — and chunk = ceil(n / grid) rows per workgroup held in LDS.
extern "C" int ksim_persistent_config(int64_t n, int* grid, int* lds_rows) {
  int g = num_cus();
  if (g <= 0 || n <= 0) return 0;
  if (g > 64 * MAXB) g = 64 * MAXB;
  if (n < (int64_t)g * 64) g = (int)((n + 63) / 64);  // >= 64 rows per workgroup
  // tables the dual-hypothesis split covers in 64 workgroups (<= 192 rows each) take 64: one
  // workgroup per sweep lane (fewer granules per lane on the decision's critical path)
  if (g > 64 && n <= 64 * 192) g = 64;
  if (const char* e = getenv("KSIM_PERSIST_GRID")) {  // diagnostic cap (grid A/B)
    const int cap = atoi(e);
    if (cap > 0 && cap < g) g = cap;
  }
  if (g < 1) g = 1;
  const int64_t chunk = (n + g - 1) / g;
  if (chunk * LDS_ROW_BYTES > LDS_BUDGET || chunk > 4095 || chunk > 8 * 448) return 0;  // launch mode
  *grid = g;
  *lds_rows = (int)chunk;
  return 1;
}

extern "C" size_t ksim_persistent_granule_bytes(int) {
  return (size_t)(NSLOT * MAXG * GR + NSLOT * GR) * sizeof(uint64_t);
}

// Static LDS of the kernel instance (granule stash, rings, partials), for the dynamic budget.
template <int BS, int NPT, int MB>
static size_t static_lds() {
  hipFuncAttributes fa;
  if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(&ksim_persistent_kernel<BS, NPT, MB>)) != hipSuccess) return 48 * 1024;
  return fa.sharedSizeBytes;
}

template <int BS, int NPT, int MB>
static hipError_t launch_persistent(const KsimCtx* c, const KsimCtx* cdev, uint64_t* granules, int grid, int lds_rows,
                                    hipStream_t s) {
  const size_t lds_max = 160 * 1024 - static_lds<BS, NPT, MB>();
  auto al = [](size_t b) { return (b + 15) & ~(size_t)15; };
  size_t off = al((size_t)lds_rows * LDS_ROW_BYTES);
  if (off > lds_max) return hipErrorInvalidValue;  // ksim_persistent_config keeps rows within budget
  PLayout L{};
  // the rows' host ports, when the node table has any and they fit
  const size_t pbytes = al((size_t)lds_rows * 4) + al((size_t)lds_rows * 8 * c->port_slots);
  if (c->port_slots > 0 && off + pbytes <= lds_max) {
    L.ps = c->port_slots;
    L.off_pc = (int32_t)off;
    L.off_pk = (int32_t)(off + al((size_t)lds_rows * 4));
    off += pbytes;
  }
  // the pod-class tables, when they fit
  const size_t C = (size_t)c->n_classes_dev;
  const size_t tb = al(C * c->lwords * 4) + 2 * al(C * c->twords * 4) + al(C * c->n_taint_sets) + al(C * c->n_label_sets) +
                    3 * al(C * c->val_w * 8);
  if (C > 0 && off + tb <= lds_max) {
    L.tables = 1;
    L.off_sel = (int32_t)off; off += al(C * c->lwords * 4);
    L.off_tok = (int32_t)off; off += al(C * c->twords * 4);
    L.off_nok = (int32_t)off; off += al(C * c->twords * 4);
    L.off_ttc = (int32_t)off; off += al(C * c->n_taint_sets);
    L.off_nac = (int32_t)off; off += al(C * c->n_label_sets);
    L.off_ttv = (int32_t)off; off += al(C * c->val_w * 8);
    L.off_nav = (int32_t)off; off += al(C * c->val_w * 8);
    L.off_nad = (int32_t)off; off += al(C * c->val_w * 8);
    const size_t sb = al(C * (size_t)lds_rows * 2);
    if (off + sb <= lds_max && !getenv("KSIM_NO_STATIC_TABLE")) {
      L.off_st = (int32_t)off;
      off += sb;
    }
  }
  hipError_t e = ksim_check_coresident(ksim_persistent_kernel<BS, NPT, MB>, grid, BS, off);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL((ksim_persistent_kernel<BS, NPT, MB>), dim3(grid), dim3(BS), off, s, *c, cdev, granules, L);
  return hipGetLastError();
}

extern "C" hipError_t ksim_launch_persistent(const KsimCtx* c, const KsimCtx* cdev, uint64_t* granules, int grid,
                                             int lds_rows, hipStream_t s) {
  if (grid <= 64 && lds_rows <= 448) return launch_persistent<512, 1, 1>(c, cdev, granules, grid, lds_rows, s);
  if (lds_rows <= 448) return launch_persistent<512, 1, MAXB>(c, cdev, granules, grid, lds_rows, s);
  if (lds_rows <= 896) return launch_persistent<512, 2, MAXB>(c, cdev, granules, grid, lds_rows, s);
  if (lds_rows <= 1792) return launch_persistent<512, 4, MAXB>(c, cdev, granules, grid, lds_rows, s);
  return launch_persistent<512, 8, MAXB>(c, cdev, granules, grid, lds_rows, s);
}

extern "C" int ksim_selftest(void) {
  int32_t* d = nullptr;
  const int nb = 4;
  if (hipMalloc(&d, nb * 3 * 64 * sizeof(int32_t)) != hipSuccess) return -1;
  hipLaunchKernelGGL(ksim_wave_selftest_kernel, dim3(nb), dim3(64), 0, 0, d);
  int32_t h[nb * 3 * 64];
  int bad = -1;
  if (hipDeviceSynchronize() == hipSuccess && hipMemcpy(h, d, sizeof h, hipMemcpyDeviceToHost) == hipSuccess) {
    bad = 0;
    for (int b = 0; b < nb; ++b) {
      int32_t v[64], mx = INT32_MIN, sum = 0, pre = 0;
      for (int l = 0; l < 64; ++l) {
        v[l] = (int32_t)((l * 7919 + 13) % 97) - 40 + b * 11;
        mx = v[l] > mx ? v[l] : mx;
        sum += v[l];
      }
      for (int l = 0; l < 64; ++l) {
        pre += v[l];
        bad += h[(b * 3 + 0) * 64 + l] != mx;
        bad += h[(b * 3 + 1) * 64 + l] != sum;
        bad += h[(b * 3 + 2) * 64 + l] != pre;
      }
    }
  }
  (void)hipFree(d);
  return bad;
}
