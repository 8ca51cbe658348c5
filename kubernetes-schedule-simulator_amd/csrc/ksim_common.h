// ksim_common.h — device-side data layout and the per-node predicate/priority evaluation
// shared by the launch-mode and persistent kernels (gfx950 / CDNA4, wave64).
//
// One node per lane.  Everything a resource-only pod reads per node is the 60-byte
// "row": alloc cpu/mem, requested cpu/mem, non-zero requested cpu/mem (6 x i64),
// allowed pods + pod count (2 x i32) and the flags word (u32) that carries both the
// static condition bits and the library-maintained "gpu/ephemeral already
// over-committed" bits, so pods that request no gpu/ephemeral storage never read those
// columns (PodFitsResources compares alloc < podReq + requested even for a zero
// request, predicates.go:739-751).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/ksim.h"

#define KSIM_BLOCK 256
#define KSIM_WAVES (KSIM_BLOCK / 64)

// predicate reasons that are copied straight from the node condition bits
#define KSIM_COND_REASON_MASK (KSIM_N_NOT_READY | KSIM_N_OUT_OF_DISK | KSIM_N_NET_UNAVAIL | KSIM_N_UNSCHEDULABLE)

struct __attribute__((aligned(16))) KsimPartial {
  int64_t mx[KSIM_MAX_RCLASS];   // max map score among fit nodes of each reduce class
  int32_t cnt[KSIM_MAX_RCLASS];  // nodes at that max
  int32_t fit;                   // fit nodes in the block
  int32_t pad[3];
  int32_t hist[KSIM_NREASONS];   // failure reasons (only when collecting)
};

// Per-block candidate masks of the launch-form scan, beside the partials: for every reduce class q
// and node slot k of the chunk, each wave's ballot of its nodes at the wave's maximum of class q
// ([q][k][wave], q = KSIM_MAX_RCLASS: the fit ballot), then each wave's maximum per class.  The
// last block picks the node from the chosen block's masks instead of re-evaluating that block.
#define KSIM_PM_NPT 8
#define KSIM_PM_MASK(q, k, w) ((((q) * KSIM_PM_NPT) + (k)) * KSIM_WAVES + (w))
#define KSIM_PM_MX(q, w) ((KSIM_MAX_RCLASS + 1) * KSIM_PM_NPT * KSIM_WAVES + (q) * KSIM_WAVES + (w))
#define KSIM_PM_STRIDE ((KSIM_MAX_RCLASS + 1) * KSIM_PM_NPT * KSIM_WAVES + KSIM_MAX_RCLASS * KSIM_WAVES)

// Inter-pod affinity tables on the device (ksim_load_affinity; layout in include/ksim.h).
struct KsimAff {
  int64_t n;                       // nodes (the dom stride)
  const int32_t* __restrict__ dom; // [n_keys][n]
  const uint64_t* __restrict__ ident_sel;
  const uint64_t* __restrict__ ident_anti;
  const uint64_t* __restrict__ ident_prio;
  const int32_t* __restrict__ pair_sel;
  const int32_t* __restrict__ pair_key;
  const int64_t* __restrict__ pair_off;
  const int32_t* __restrict__ carry_key;
  const int64_t* __restrict__ carry_off;
  const int32_t* __restrict__ ac;  // [n_aclass][6]
  const ksim_aff_term* __restrict__ terms;
  const ksim_aff_carry* __restrict__ carries;
  int32_t* cnt;                    // counted pairs, per domain
  int64_t* carried;                // carried terms, per domain
  int64_t* mm;                     // pass A results: [0..1] min / max of the raw InterPodAffinity sums,
                                   // [2] SelectorSpread maxCountByNodeName, [3] haveZones, [4] maxCountByZone
  int64_t* part;                   // [grid][4] pass A block partials
  uint32_t* ticket;                // pass A arrival counter
  const int32_t* __restrict__ spread_pair;  // [n_aclass] or null
  int64_t* zsum;                   // [n_zone] SelectorSpread countsByZone being summed (pass A, zeroed by it)
  int64_t* zread;                  // [n_zone] countsByZone of the current pod (read by the scan)
  int32_t n_pair;
  int32_t sel_words, carry_words;
  int32_t zone_key;                // -1: no zone key
  int32_t n_zone;
  int32_t pad;
  // the auxiliary counted priority (ksim_affinity_tables.aux_*; launch form only), aux_pair null: none.
  // Pass A adds mm[5] max count, mm[6] summed count, mm[7] haveZones, mm[8] max domain sum over the
  // fit nodes, and per aux_key domain the fit nodes' summed counts (asum → aread, as zsum / zread)
  const int32_t* __restrict__ aux_pair;  // [n_aclass]
  int64_t* asum;
  int64_t* aread;
  int64_t aux_w;
  int32_t aux_key, aux_kind, n_adom, pad2;
  // CheckServiceAffinity's lender agreement (ksim_affinity_tables.svc_*; launch form only), svc_class
  // null: none.  svc_conflict is device-mutable (the commits' disagreement bits); err bit 128 = a pod
  // read a disagreeing label (the host refuses the run)
  const int32_t* __restrict__ svc_class;
  const uint32_t* __restrict__ svc_miss;
  const ksim_svc_ident* __restrict__ svc;
  uint32_t* svc_conflict;
  const int32_t* __restrict__ svc_of_off;
  const int32_t* __restrict__ svc_of;
  int32_t n_svc, n_svc_labels;
};

#define KSIM_AFF_MM 9      // pass-A result words
// node-sharded launch form: exchange slots (pod mod KSIM_LX_SLOTS) of KSIM_LX_REC words per rank,
// each word (tag:24 | value:40): the fit count, then per reduce class its max (biased by 2^39) and count
#define KSIM_LX_SLOTS 4
#define KSIM_LX_REC (1 + 2 * KSIM_MAX_RCLASS)
#define KSIM_LX_BIAS (1ll << 39)
// ... and pass A's (after the launch region): min / max raw InterPodAffinity sum, max spread count,
// haveZones, then the zone sums (<= KSIM_PX_ZONES zones), same word format
#define KSIM_PX_ZONES 24
#define KSIM_PX_ADOMS 24  // the auxiliary priority's domains: its max / sum / haveZones and domain sums follow the zones
#define KSIM_PX_REC (4 + KSIM_PX_ZONES + 3 + KSIM_PX_ADOMS)
#define KSIM_AFF_PART 8    // pass-A block-partial words

// Volume tables on the device (ksim_load_volumes; layout in include/ksim.h).
struct KsimVol {
  int64_t n;                            // nodes (the slot stride)
  uint64_t* slots;                      // [vol_slots][n] KSIM_VOL_SLOT words
  int32_t* slot_count;                  // [n]
  const uint32_t* __restrict__ key_filter;
  const int32_t* __restrict__ vc;       // [n_vclass][2]
  const uint32_t* __restrict__ vc_filter;
  const ksim_vol_ref* __restrict__ refs;
  const uint32_t* __restrict__ zone_ok; // [n_vclass][zone_words] or null
  int32_t max_vols[3];
  int32_t vol_slots;
  int32_t zone_words;
  int32_t pad;
};

// Result block of the per-pod drop-in entry points (int32 words; pinned host memory mapped into the
// device's address space, written by the scan / assume kernels, read by the host after the sync).
#define KSIM_RES_NODE 0
#define KSIM_RES_FIT 1
#define KSIM_RES_STATUS 2   /* bit 0: a committed quantity left the fast kernels' exact range */
#define KSIM_RES_ERR 3      /* the sticky device error word after the call */
#define KSIM_RES_REASONS 4
#define KSIM_RES_CTR (KSIM_RES_REASONS + KSIM_NREASONS)  /* uint64 lastNodeIndex after the call */
#define KSIM_RES_WORDS (KSIM_RES_CTR + 2)
#define KSIM_ONE_PORTS 16  // host ports a per-pod launch carries in its kernel arguments
// per-pod pick kernel (ksim_pick_kernel): <= 64 blocks, each publishing a pass-A record (min /
// max raw InterPodAffinity sum, SelectorSpread max count, haveZones, <= 60 zone sums) and a
// decision record (fit count, per reduce class max map score and count, reasons when it fits
// nothing), 8-byte words tag:8 | value:56
#define KSIM_PICK_MAXG 64
#define KSIM_PICK_ZMAX 60
#define KSIM_PICK_RA (4 + KSIM_PICK_ZMAX)
#define KSIM_PICK_RB (1 + 2 * KSIM_MAX_RCLASS + KSIM_NREASONS)
#define KSIM_PICK_WORDS (KSIM_PICK_MAXG * (KSIM_PICK_RA + KSIM_PICK_RB))  /* one record buffer (two are allocated) */

struct KsimCtx {
  // ---- node table (name-rank order) ----
  int64_t n;
  const int64_t* __restrict__ alloc_cpu;
  const int64_t* __restrict__ alloc_mem;
  const int64_t* __restrict__ alloc_gpu;
  const int64_t* __restrict__ alloc_eph;
  const int32_t* __restrict__ allowed_pods;
  uint32_t* flags;
  const int32_t* __restrict__ label_set;
  const int32_t* __restrict__ taint_set;
  const int64_t* __restrict__ alloc_scalar;
  int64_t* req_cpu;
  int64_t* req_mem;
  int64_t* req_gpu;
  int64_t* req_eph;
  int64_t* nz_cpu;
  int64_t* nz_mem;
  int32_t* pod_count;
  int64_t* req_scalar;
  uint64_t* ports;       // slot-major [port_slots][n]
  int32_t* port_count;
  int32_t port_slots;
  int32_t n_scalar;
  // ---- pod-class tables ----
  const uint32_t* __restrict__ sel_ok;
  const uint32_t* __restrict__ taint_ok;
  const uint32_t* __restrict__ noexec_ok;
  const uint8_t* __restrict__ tt_class;
  const uint8_t* __restrict__ na_class;
  const int32_t* __restrict__ n_tt;
  const int32_t* __restrict__ n_na;
  const int64_t* __restrict__ tt_val;
  const int64_t* __restrict__ na_val;
  const int64_t* __restrict__ na_add;  // [C][KSIM_MAX_RCLASS] weighted per-NA-class addend, or null
  const uint32_t* __restrict__ svc_ok; // [C][lwords] CheckServiceAffinity per label set, or null
  int32_t use_na;                      // NA class dimension in use: NodeAffinity weight or na_add
  int32_t lwords, twords, n_label_sets, n_taint_sets;
  int32_t val_w;          // row width of tt_val / na_val / na_add (ksim_class_tables.val_width, >= 16)
  int32_t n_classes_dev;  // pod classes in the tables
  int32_t fuse_a;         // launch form: pass A fused into the scan (grid barrier; co-resident grid)
  uint64_t barrier_ticks; // fused pass A: bound of the grid-barrier wait (s_memrealtime ticks, 100 MHz)
  // ---- pod queue ----
  const ksim_pod* __restrict__ pods;
  const uint64_t* __restrict__ pod_ports;
  const ksim_scalar_req* __restrict__ pod_scalars;
  // ---- configuration ----
  uint32_t preds;
  int32_t no_prio;
  int32_t collect;
  int32_t no_commit;      // 1: decide only (genericScheduler.Schedule without Scheduler.assume)
  int64_t w[KSIM_NW];
  // ---- run state ----
  int64_t* cursor;        // next pod to schedule (device)
  int64_t first, end;     // [first, end) of this call
  uint64_t* counter;      // genericScheduler.lastNodeIndex
  uint32_t* ticket;       // last-block arrival counter
  KsimPartial* partials;  // [grid]
  int64_t* wmx;           // wide reduce classes (K > KSIM_MAX_RCLASS, launch form): per block and class the
  int32_t* wcnt;          // max map score among its fit nodes and their count, [grid][KSIM_MAX_WIDE]
  uint64_t* pmask;        // [grid][KSIM_PM_STRIDE] candidate masks (KSIM_PM_*)
  uint64_t* pick;         // per-pod pick kernel: the blocks' tagged exchange records (KSIM_PICK_*)
  int32_t* out_node;      // [end-first]
  int32_t* out_reasons;   // [end-first][KSIM_NREASONS]
  int32_t* err;           // sticky error word
  int64_t chunk;          // nodes per block
  uint64_t* dbg;          // diagnostic stamp sums (KSIM_STAMPS builds only), else null
  int32_t* out_fit;       // optional (per-pod drop-in): [0] = len(filtered), [1] |= ksim_row_status
  const KsimAff* aff;     // inter-pod affinity tables (device), null when none are loaded
  const KsimVol* vol;     // volume tables (device), null when none are loaded
  // node-sharded launch form (world > 1, pods the fast kernel does not take; SURVEY.md §8e Phase A):
  // the last block exchanges this rank's fit count and per-class (max, count) with every rank
  // through the launch region of the exchange buffers, decides on the world's, and the rank that
  // holds the selected node commits it.  sh_world 0: off
  int32_t sh_world, sh_rank;
  int64_t sh_base;                       // global name rank of this shard's first node
  uint32_t sh_tag0;                      // tag of pod p: 1 + (sh_tag0 + p - first) mod (2^24 - 1)
  uint32_t sh_pad;
  uint64_t sh_start_ticks;               // the first pod's wait bound (the start handshake)
  uint64_t* sh_peers[KSIM_MAX_RANKS];    // every rank's launch region as mapped here (self included)
  // per-pod launches (ksim_schedule_one): the pod and its arrays travel in the kernel arguments,
  // so no read of host memory or of a staging copy sits on the kernel's critical path
  int32_t one;            // 1: the pod is one_pod (index first), its ports / scalars one_ports / one_scalars
  uint32_t pick_tag;      // per-pod pick kernel: this call's record tag (1..255)
  ksim_pod one_pod;
  uint64_t one_ports[KSIM_ONE_PORTS];
  ksim_scalar_req one_scalars[KSIM_MAX_SCALAR];
};
// KsimCtx is passed BY VALUE as the launch-form kernels' argument: it must stay within the
// kernel-argument segment (4 KiB on gfx950; a larger struct makes hipLaunchKernel fail with
// "invalid argument" — the round-4 r4b failure mode while the per-pod fields were being added).
static_assert(sizeof(KsimCtx) <= 4096 - 64, "KsimCtx exceeds the kernel-argument limit");

// The pod of a launch and its arrays (KsimCtx::one: the kernel arguments).
__device__ __forceinline__ uint64_t ksim_pod_port(const KsimCtx& c, const ksim_pod& P, int32_t k) {
  return c.one ? c.one_ports[k] : c.pod_ports[P.port_off + k];
}
__device__ __forceinline__ ksim_scalar_req ksim_pod_scalar(const KsimCtx& c, const ksim_pod& P, int32_t s) {
  return c.one ? c.one_scalars[s] : c.pod_scalars[P.scalar_off + s];
}

// The resident per-pod service's mailbox (ksim_serve_kernel), in coherent host memory mapped
// into the device.  A message is KSIM_SERVE_MSG_WORDS 32-bit payload words, each stored by the
// host as one 8-byte word `payload | (uint32)seq << 32`: the device reads the whole message with
// one 16-byte load per lane (one PCIe round trip) and takes it when every word carries the
// message's number — no separate sequence word, no second round trip for the body.  The answer
// travels the same way: every result word the block that answers writes is one 8-byte store
// `value | (uint32)seq << 32`, and the host accepts an answer only when every word it reads
// carries its message's number, so a word of an earlier answer can never be taken for this one
// (no completion flag, no ordering between the words needed).
#define KSIM_SERVE_EXIT 0
#define KSIM_SERVE_SCHEDULE 1
#define KSIM_SERVE_ASSUME 2
#define KSIM_SERVE_UNDO 3   // undo a tentative commit of shared state (below); answered by the node's block
#define KSIM_SERVE_SYNC_ACQUIRE 1  // the previous message committed state other blocks read: acquire first
#define KSIM_SERVE_MSG_WORDS 128
// payload word offsets
#define KSIM_SERVE_W_TYPE 0      // KSIM_SERVE_*
#define KSIM_SERVE_W_NOCOMMIT 1  // SCHEDULE: 1 = decide only
#define KSIM_SERVE_W_TAG 2       // SCHEDULE: the pick records' tag (1..254; its parity picks the record buffer)
#define KSIM_SERVE_W_SYNC 3      // KSIM_SERVE_SYNC_* (the host knows which pods commit shared counts)
#define KSIM_SERVE_W_NODE 4      // ASSUME: the node (two words, low first)
#define KSIM_SERVE_W_POD 6       // ksim_pod (32 words)
#define KSIM_SERVE_W_PORTS (KSIM_SERVE_W_POD + (int)(sizeof(ksim_pod) / 4))   // KSIM_ONE_PORTS keys
#define KSIM_SERVE_W_SCALARS (KSIM_SERVE_W_PORTS + 2 * KSIM_ONE_PORTS)       // KSIM_MAX_SCALAR requests
// Every message (EXIT included) also says what became of the last tentative commit (below): the
// message number of its SCHEDULE and KSIM_TENT_* (the block holding its record acts on the first
// message it takes after the host decided)
#define KSIM_SERVE_W_TENT_SEQ 120
#define KSIM_SERVE_W_TENT_ACT 121
#define KSIM_TENT_NONE 0     // undecided (the record stays)
#define KSIM_TENT_CONFIRM 1  // AssumePod named the same pod and node: the commit stands, drop the record
#define KSIM_TENT_UNDO 2     // anything else came first: undo the commit, then drop the record
// SCHEDULE's KSIM_SERVE_W_NOCOMMIT: 0 commit (SCHEDULE_ASSUME), 1 decide only, 2 tentative commit
// (SCHEDULE_ONLY: the owner block commits it and keeps a record, and answers the row's port count
// and flags before the commit in the first two reason words, so the host can undo it without the
// kernel too).  A commit of the pod's row alone is undone by the record's block before it reads
// the row again (any later message carries the decision); a commit of state other blocks read
// (volume mounts, inter-pod affinity / SelectorSpread counts) is undone by an UNDO message of its
// own, answered after the undo is released, and the next message acquires.
#define KSIM_SERVE_TENTATIVE 2
static_assert(sizeof(ksim_pod) % 4 == 0 && sizeof(ksim_scalar_req) % 4 == 0, "mailbox words");
static_assert(KSIM_SERVE_W_SCALARS + (int)(KSIM_MAX_SCALAR * sizeof(ksim_scalar_req) / 4) <= KSIM_SERVE_W_TENT_SEQ,
              "a mailbox message holds a pod with KSIM_ONE_PORTS ports and KSIM_MAX_SCALAR scalars");
// Leaving.  The grid leaves on an EXIT message, or by agreement when idle: a block that has seen
// no message for idle_ticks votes in a device word (KSIM_SERVE_ST_*, agent-scope CAS); the vote
// that would make it unanimous instead sets LEFT, and a block that has voted takes a newly seen
// message only after a veto (a CAS that bumps the epoch and clears the votes), which fails once
// LEFT is set.  A block that has not voted never checks: LEFT needs its vote.  So a message is
// taken by every block or by none, and a grid that left by agreement answered everything it took;
// the LEFT voter then stores `left = launch id << 32 | last message` so the host knows that its
// unanswered message was never taken and relaunches the kernel to serve it (ksim_cache.cpp).
#define KSIM_SERVE_ST_LEFT (1ull << 63)
#define KSIM_SERVE_ST_VOTES(s) ((uint32_t)((s) & 0xffffu))
#define KSIM_SERVE_ST_EPOCH(s) ((uint32_t)(((s) >> 16) & 0xffffffffu))
#define KSIM_SERVE_ST_MAKE(epoch, votes) ((((uint64_t)(uint32_t)(epoch)) << 16) | (uint64_t)(votes))
struct KsimServeBox {
  uint64_t msg[KSIM_SERVE_MSG_WORDS];  // host: the current message (16-byte aligned)
  uint64_t ans[KSIM_RES_WORDS];        // device: the answer, word k = KSIM_RES_* word | seq << 32
  uint64_t left;                       // device: launch id << 32 | last message, when it left by agreement
  uint64_t undo_ack;                   // device: the tentative commit (its message number) last undone
  uint64_t pad1[6];
};
// A tentative commit as the resident kernel's owner block records it (LDS) and as the host keeps
// it (to undo it with ksim_launch_undo when the kernel that holds the record is gone).
struct KsimTentRec {
  int64_t node;
  uint32_t seq;
  int32_t valid;
  int32_t cnt0;  // the row's port count before the commit (the commit appends its new keys)
  uint32_t fl0;  // the row's flags before the commit
  ksim_pod P;
  ksim_scalar_req sc[KSIM_MAX_SCALAR];
};
// The resident kernel's launch arguments beside the context.
struct KsimServeArgs {
  KsimServeBox* box;
  uint64_t* state;      // device word: the idle vote (KSIM_SERVE_ST_*), zeroed before every launch
  uint64_t seq0;        // the newest message number already handled (the kernel takes later ones)
  uint64_t idle_ticks;  // a block votes to leave after this long without a message (s_memrealtime, 100 MHz)
  uint64_t ctr0;        // lastNodeIndex as the host last saw it ...
  uint32_t ctr0_valid;  // ... when the host knows it (else the kernel reads *c.counter, coherently)
  uint32_t launch_id;
};

// Node-sharded mode (ksim_shard_*): this rank's place in the world and every rank's exchange
// buffer as mapped on this device.
struct KsimShard {
  int32_t rank, world;
  int64_t node_base;
  uint32_t xtag_base;
  uint64_t* xchg;
  uint64_t* peers[KSIM_MAX_RANKS];
  // bound of the first pod's cross-rank wait of a call (s_memrealtime ticks, 100 MHz): the start
  // handshake absorbs per-rank launch skew (first code-object load, ingest, a descheduled host
  // process); later pods keep the 2 s per-pod bound
  uint64_t start_ticks;
};

// The persistent kernels spin on each other's progress, so every workgroup of the grid must be
// resident at once: check the occupancy of this kernel at this block size and dynamic LDS on the
// current device before launching.  hipErrorCooperativeLaunchTooLarge when the grid cannot be
// co-resident (the runtime then takes the launch form, or fails in KSIM_MODE_PERSISTENT).
template <class K>
static hipError_t ksim_check_coresident(K kernel, int grid, int block, size_t lds) {
  int dev = 0, cus = 0, per_cu = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e == hipSuccess) e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, lds);
  if (e != hipSuccess) return e;
  return (int64_t)per_cu * cus >= grid ? hipSuccess : hipErrorCooperativeLaunchTooLarge;
}

// ((a*10)/b) with Go int64 semantics (wrapping multiply, truncating divide), b > 0.
// Quotients here are 0..10, so for a < 2^49 a correctly rounded double divide plus one
// integer correction is exact; larger values take the native (slow) 64-bit divide.
// The emulated 64-bit divide is ~100 instructions: kept out of line so the evaluations that
// inline ksim_mul10_div stay small (instruction-cache footprint of the persistent kernels).
__device__ __noinline__ int64_t ksim_mul10_div_slow(int64_t a, int64_t b) {
  const int64_t x = (int64_t)((uint64_t)a * 10ull);
  return x / b;
}

__device__ __forceinline__ int64_t ksim_mul10_div(int64_t a, int64_t b) {
  if (a >= 0 && a < (int64_t(1) << 49) && b > 0) {
    const int64_t x = a * 10;
    int64_t q = (int64_t)((double)x / (double)b);
    if (q * b > x) q -= 1;
    else if ((q + 1) * b <= x) q += 1;
    return q;
  }
  return ksim_mul10_div_slow(a, b);
}

// least_requested.go:44-53
__device__ __forceinline__ int64_t ksim_least(int64_t req, int64_t cap) {
  if (cap == 0 || req > cap) return 0;
  return ksim_mul10_div(cap - req, cap);
}
// most_requested.go:45-55
__device__ __forceinline__ int64_t ksim_most(int64_t req, int64_t cap) {
  if (cap == 0 || req > cap) return 0;
  return ksim_mul10_div(req, cap);
}
// balanced_resource_allocation.go:39-61 — IEEE f64, compiled with -ffp-contract=off
__device__ __forceinline__ int64_t ksim_balanced(int64_t rc, int64_t cc, int64_t rm, int64_t cm) {
  const double fc = cc == 0 ? 1.0 : (double)rc / (double)cc;
  const double fm = cm == 0 ? 1.0 : (double)rm / (double)cm;
  if (fc >= 1.0 || fm >= 1.0) return 0;
  const double diff = fabs(fc - fm);
  return (int64_t)((1.0 - diff) * 10.0);
}

__device__ __forceinline__ bool ksim_bit(const uint32_t* tab, int64_t row, int32_t words, int32_t idx) {
  return (tab[row * words + (idx >> 5)] >> (idx & 31)) & 1u;
}

// HostPortInfo.CheckConflict (pkg/scheduler/util/utils.go:101-130) against one node.
__device__ __forceinline__ bool ksim_port_conflict(const KsimCtx& c, int64_t i, uint64_t want) {
  const int32_t cnt = c.port_count[i];
  const uint32_t wip = (uint32_t)(want >> 40);
  const uint64_t wpp = want & 0xFFFFFFFFFFull;  // proto + port
  for (int32_t s = 0; s < cnt; ++s) {
    const uint64_t e = c.ports[(int64_t)s * c.n + i];
    if ((e & 0xFFFFFFFFFFull) != wpp) continue;
    const uint32_t eip = (uint32_t)(e >> 40);
    if (wip == 0 || eip == 0 || eip == wip) return true;
  }
  return false;
}

// One node's row, loaded up front so the loads issue together.
struct KsimRow {
  int64_t ac, am, rc, rm, zc, zm;
  int32_t allowed, count;
  uint32_t fl;
};

__device__ __forceinline__ KsimRow ksim_load_row(const KsimCtx& c, int64_t i) {
  KsimRow r;
  r.ac = c.alloc_cpu[i];
  r.am = c.alloc_mem[i];
  r.rc = c.req_cpu[i];
  r.rm = c.req_mem[i];
  r.zc = c.nz_cpu[i];
  r.zm = c.nz_mem[i];
  r.allowed = c.allowed_pods[i];
  r.count = c.pod_count[i];
  r.fl = c.flags[i];
  return r;
}

// PodFitsResources (predicates.go:706-778) reason mask.
__device__ __forceinline__ uint32_t ksim_resources(const KsimCtx& c, const ksim_pod& P, int64_t i,
                                                   const KsimRow& r) {
  uint32_t m = 0;
  if (r.count + 1 > r.allowed) m |= 1u << KSIM_R_INSUFFICIENT_PODS;
  if (!(P.flags & KSIM_POD_ANY_REQUEST)) return m;
  if (r.ac < P.req_cpu + r.rc) m |= 1u << KSIM_R_INSUFFICIENT_CPU;
  if (r.am < P.req_mem + r.rm) m |= 1u << KSIM_R_INSUFFICIENT_MEMORY;
  if (P.req_gpu == 0) {
    if (r.fl & KSIM_N_GPU_OVER) m |= 1u << KSIM_R_INSUFFICIENT_GPU;
  } else if (c.alloc_gpu[i] < P.req_gpu + c.req_gpu[i]) {
    m |= 1u << KSIM_R_INSUFFICIENT_GPU;
  }
  if (P.req_eph == 0) {
    if (r.fl & KSIM_N_EPH_OVER) m |= 1u << KSIM_R_INSUFFICIENT_EPHEMERAL;
  } else if (c.alloc_eph[i] < P.req_eph + c.req_eph[i]) {
    m |= 1u << KSIM_R_INSUFFICIENT_EPHEMERAL;
  }
  for (int32_t s = 0; s < P.scalar_cnt; ++s) {
    const ksim_scalar_req q = ksim_pod_scalar(c, P, s);
    const int64_t off = (int64_t)q.col * c.n + i;
    if (c.alloc_scalar[off] < q.req + c.req_scalar[off]) m |= 1u << (KSIM_R_INSUFFICIENT_SCALAR0 + q.col);
  }
  return m;
}

__device__ __forceinline__ uint32_t ksim_hostname(const ksim_pod& P, int64_t i) {
  return (P.host == -1 || P.host == i) ? 0u : (1u << KSIM_R_HOSTNAME);
}

// Where a general evaluation reads what is not in the 60-byte row: the node's label / taint
// set and host ports, the pod class's selector / toleration bits and reduce-class bytes.  This
// accessor reads the HBM table (launch mode, evaluate); the persistent kernel supplies one that
// reads its LDS-staged copies (ksim_persistent.hip), so its row waves issue no global loads.
struct KsimGlobalAcc {
  const KsimCtx& c;
  __device__ __forceinline__ bool sel_ok(const ksim_pod& P, int64_t i) const {
    return ksim_bit(c.sel_ok, P.cls, c.lwords, c.label_set[i]);
  }
  __device__ __forceinline__ bool taint_ok(const ksim_pod& P, int64_t i) const {
    return ksim_bit(c.taint_ok, P.cls, c.twords, c.taint_set[i]);
  }
  __device__ __forceinline__ bool noexec_ok(const ksim_pod& P, int64_t i) const {
    return ksim_bit(c.noexec_ok, P.cls, c.twords, c.taint_set[i]);
  }
  __device__ __forceinline__ bool port_conflict(int64_t i, uint64_t want) const { return ksim_port_conflict(c, i, want); }
  // k-th host-port key the pod wants
  __device__ __forceinline__ uint64_t want(const ksim_pod& P, int32_t k) const { return ksim_pod_port(c, P, k); }
  __device__ __forceinline__ int tt_class(const ksim_pod& P, int64_t i) const {
    return c.tt_class[(int64_t)P.cls * c.n_taint_sets + c.taint_set[i]];
  }
  __device__ __forceinline__ int na_class(const ksim_pod& P, int64_t i) const {
    return c.na_class[(int64_t)P.cls * c.n_label_sets + c.label_set[i]];
  }
};

template <class A>
__device__ __forceinline__ uint32_t ksim_hostports(const KsimCtx& c, const ksim_pod& P, int64_t i, const A& a) {
  for (int32_t k = 0; k < P.port_cnt; ++k)
    if (a.port_conflict(i, a.want(P, k))) return 1u << KSIM_R_HOST_PORTS;
  return 0;
}

template <class A>
__device__ __forceinline__ uint32_t ksim_selector(const ksim_pod& P, int64_t i, const A& a) {
  if (!(P.flags & KSIM_POD_NEED_SELECTOR)) return 0;
  return a.sel_ok(P, i) ? 0u : (1u << KSIM_R_NODE_SELECTOR);
}

// ---- inter-pod affinity (tables: include/ksim.h, ksim/affinity.py) ----
__device__ __forceinline__ int32_t ksim_dom(const KsimAff& A, int32_t key, int64_t i) {
  return A.dom[(int64_t)key * A.n + i];
}

// A count > 0 of counted pair `pair` at node i's domain of the pair's key.
__device__ __forceinline__ bool ksim_pair_hit(const KsimAff& A, int32_t pair, int64_t i) {
  const int32_t d = ksim_dom(A, A.pair_key[pair], i);
  return d >= 0 && A.cnt[A.pair_off[pair] + d] > 0;
}

// InterPodAffinityMatches (predicates.go:1143-1160) for pod P on node i: existing pods'
// required anti-affinity terms that P matches (satisfiesExistingPodsAntiAffinity, :1340-1379),
// then P's required affinity terms (anyPodMatchesPodAffinityTerm, :1161-1194; a term nobody
// matches is waived when P matches it itself, :1405-1424), then its required anti-affinity
// terms (:1430-1441).  Reason mask, 0 = fits.  Out of line: only affinity pods call it.
__device__ __forceinline__ uint32_t ksim_interpod_pred_body(const KsimAff& A, const ksim_pod& P, int64_t i) {
  const uint32_t base = 1u << KSIM_R_POD_AFFINITY;
  if (P.aff_ident > 0) {
    const uint64_t* mw = A.ident_anti + (int64_t)(P.aff_ident - 1) * A.carry_words;
    for (int32_t w = 0; w < A.carry_words; ++w) {
      uint64_t m = mw[w];
      while (m) {
        const int e = 64 * w + __builtin_ctzll(m);
        m &= m - 1;
        const int32_t d = ksim_dom(A, A.carry_key[e], i);
        if (d >= 0 && A.carried[A.carry_off[e] + d] > 0) return base | (1u << KSIM_R_EXISTING_ANTI_AFFINITY);
      }
    }
  }
  if (P.aff_class <= 0) return 0;
  const int32_t* ac = A.ac + 6 * (int64_t)(P.aff_class - 1);
  for (int32_t j = ac[0], e = ac[0] + ac[1]; j < e; ++j) {
    const ksim_aff_term t = A.terms[j];
    const bool match = ksim_dom(A, t.gate_key, i) >= 0 && ksim_pair_hit(A, t.pair, i);
    if (t.kind == KSIM_AFF_REQ_AFFINITY) {
      if (!match && (!t.self_ok || ksim_pair_hit(A, t.exist_pair, i))) return base | (1u << KSIM_R_AFFINITY_RULES);
    } else if (match) {
      return base | (1u << KSIM_R_ANTI_AFFINITY_RULES);
    }
  }
  return 0;
}
__device__ __noinline__ uint32_t ksim_interpod_pred(const KsimAff& A, const ksim_pod& P, int64_t i) { return ksim_interpod_pred_body(A, P, i); }

// Does pod P read the InterPodAffinity priority (own preferred terms, or carried priority
// terms its identity matches)?
__device__ __forceinline__ bool ksim_interpod_prio_work(const KsimAff& A, const ksim_pod& P) {
  if (P.aff_class > 0 && A.ac[6 * (int64_t)(P.aff_class - 1) + 3] > 0) return true;
  if (P.aff_ident <= 0) return false;
  const uint64_t* mw = A.ident_prio + (int64_t)(P.aff_ident - 1) * A.carry_words;
  for (int32_t w = 0; w < A.carry_words; ++w)
    if (mw[w]) return true;
  return false;
}

// CalculateInterPodAffinityPriority's per-node sum (interpod_affinity.go:124-214) before
// normalisation: P's preferred terms weight the placed pods they match in the node's domain,
// the carried terms of placed pods P matches add their per-domain amounts.
__device__ __forceinline__ int64_t ksim_interpod_raw_body(const KsimAff& A, const ksim_pod& P, int64_t i) {
  int64_t s = 0;
  if (P.aff_class > 0) {
    const int32_t* ac = A.ac + 6 * (int64_t)(P.aff_class - 1);
    for (int32_t j = ac[2], e = ac[2] + ac[3]; j < e; ++j) {
      const ksim_aff_term t = A.terms[j];
      const int32_t d = ksim_dom(A, A.pair_key[t.pair], i);
      if (d >= 0) s += t.weight * (int64_t)A.cnt[A.pair_off[t.pair] + d];
    }
  }
  if (P.aff_ident > 0) {
    const uint64_t* mw = A.ident_prio + (int64_t)(P.aff_ident - 1) * A.carry_words;
    for (int32_t w = 0; w < A.carry_words; ++w) {
      uint64_t m = mw[w];
      while (m) {
        const int e = 64 * w + __builtin_ctzll(m);
        m &= m - 1;
        const int32_t d = ksim_dom(A, A.carry_key[e], i);
        if (d >= 0) s += A.carried[A.carry_off[e] + d];
      }
    }
  }
  return s;
}
__device__ __noinline__ int64_t ksim_interpod_raw(const KsimAff& A, const ksim_pod& P, int64_t i) { return ksim_interpod_raw_body(A, P, i); }

// fScore = MaxPriority * ((count - min) / (max - min)) in float64, truncated (:228-236); the
// counts are integers below 2^53, so the float64 operands are exact as in Go.
__device__ __forceinline__ int64_t ksim_interpod_score(int64_t raw, int64_t mn, int64_t mx) {
  if (mx - mn <= 0) return 0;
  return (int64_t)(10.0 * ((double)(raw - mn) / (double)(mx - mn)));
}

// NodeInfo.AddPod / RemovePod of an affinity pod on node w (sign +1 / -1): every counted pair
// whose selector its identity matches, and the amounts of the terms it carries.  Single thread.
__device__ __forceinline__ void ksim_aff_commit_body(const KsimAff& A, const ksim_pod& P, int64_t w, int32_t sign,
                                             int32_t lane = 0, int32_t stride = 1) {
  // lanes [lane, stride) split the pairs and carries; the updates are atomic adds (order-free sums)
  if (P.aff_ident > 0) {
    const uint64_t* sm = A.ident_sel + (int64_t)(P.aff_ident - 1) * A.sel_words;
    for (int32_t c = lane; c < A.n_pair; c += stride) {
      const int32_t s = A.pair_sel[c];
      if (!((sm[s >> 6] >> (s & 63)) & 1ull)) continue;
      const int32_t d = ksim_dom(A, A.pair_key[c], w);
      if (d >= 0) atomicAdd(&A.cnt[A.pair_off[c] + d], sign);
    }
  }
  if (P.aff_class > 0) {
    const int32_t* ac = A.ac + 6 * (int64_t)(P.aff_class - 1);
    for (int32_t j = ac[4] + lane, e = ac[4] + ac[5]; j < e; j += stride) {
      const ksim_aff_carry k = A.carries[j];
      const int32_t d = ksim_dom(A, A.carry_key[k.term], w);
      if (d >= 0)
        atomicAdd(reinterpret_cast<unsigned long long*>(&A.carried[A.carry_off[k.term] + d]),
                  (unsigned long long)((int64_t)sign * k.amount));
    }
  }
}
__device__ __noinline__ void ksim_aff_commit(const KsimAff& A, const ksim_pod& P, int64_t w, int32_t sign,
                                             int32_t lane = 0, int32_t stride = 1) {
  ksim_aff_commit_body(A, P, w, sign, lane, stride);
}

// The counted pair of pod P's SelectorSpread selectors, or -1.
__device__ __forceinline__ int32_t ksim_spread_pair(const KsimAff& A, const ksim_pod& P) {
  return (A.spread_pair && P.aff_class > 0) ? A.spread_pair[P.aff_class - 1] : -1;
}

// CalculateSpreadPriorityReduce's score of one fit node (selector_spreading.go:121-174) from its
// count, the pass-A maxima and the zone's summed count; float64 without contraction as in Go.
__device__ __forceinline__ int64_t ksim_spread_score(int64_t cnt, int64_t max_node, bool have_zones, int32_t zone,
                                                     int64_t zone_cnt, int64_t max_zone) {
  const double zw = 2.0 / 3.0;  // zoneWeighting (selector_spreading.go:33)
  double f = 10.0;
  if (max_node > 0) f = 10.0 * ((double)(max_node - cnt) / (double)max_node);
  if (have_zones && zone >= 0) {
    double zs = 10.0;
    if (max_zone > 0) zs = 10.0 * ((double)(max_zone - zone_cnt) / (double)max_zone);
    f = (f * (1.0 - zw)) + (zw * zs);
  }
  return (int64_t)f;
}

// The auxiliary priority's counted pair of pod P, or -1.
__device__ __forceinline__ int32_t ksim_aux_pair(const KsimAff& A, const ksim_pod& P) {
  return (A.aux_pair && P.aff_class > 0) ? A.aux_pair[P.aff_class - 1] : -1;
}

// The auxiliary priority's score of one fit node (ksim_affinity_tables.aux_*): cnt its count, d its
// aux_key domain (-1: no label), dsum the fit nodes' summed count in d; the pass-A words amx (max
// count), atot (summed count), ahz (haveZones), azmx (max domain sum).
__device__ __forceinline__ int64_t ksim_aux_score(int32_t kind, int64_t cnt, int32_t d, int64_t dsum, int64_t amx,
                                                  int64_t atot, bool ahz, int64_t azmx) {
  if (kind == KSIM_AUX_SPREAD) return ksim_spread_score(cnt, amx, ahz, d, dsum, azmx);
  // CalculateAntiAffinityPriorityReduce (selector_spreading.go:248-275): float64 as in Go
  if (d < 0) return 0;
  if (atot <= 0) return 10;
  return (int64_t)(10.0 * ((double)(atot - dsum) / (double)atot));
}

__device__ __forceinline__ bool ksim_is_aff_pod(const KsimCtx& c, const ksim_pod& P) {
  return c.aff && (P.aff_ident > 0 || P.aff_class > 0);
}

// ---- volumes (tables: include/ksim.h, ksim/volumes.py) ----
__device__ __forceinline__ bool ksim_is_vol_pod(const KsimCtx& c, const ksim_pod& P) {
  return c.vol && P.vol_class > 0;
}

// Mount counts of key k on node i: slot index or -1.
__device__ __forceinline__ int32_t ksim_vol_find(const KsimVol& V, int64_t i, int32_t cnt, int32_t key) {
  for (int32_t s = 0; s < cnt; ++s)
    if ((int32_t)(V.slots[(int64_t)s * V.n + i] >> 32) == key) return s;
  return -1;
}

// The node's mount words, all loads in flight at once (nodes with up to KSIM_VOL_REG mounted keys;
// more take the one-slot-at-a-time form): the lookups below then run on registers instead of one
// dependent load per slot.
#define KSIM_VOL_REG 16
__device__ __forceinline__ void ksim_vol_load_slots(const KsimVol& V, int64_t i, int32_t cnt, uint64_t (&sw)[KSIM_VOL_REG]) {
#pragma unroll
  for (int s = 0; s < KSIM_VOL_REG; ++s) sw[s] = s < cnt ? V.slots[(int64_t)s * V.n + i] : 0ull;
}
__device__ __forceinline__ int32_t ksim_vol_find_reg(const uint64_t (&sw)[KSIM_VOL_REG], int32_t cnt, int32_t key) {
  int32_t f = -1;
#pragma unroll
  for (int s = KSIM_VOL_REG - 1; s >= 0; --s) f = (s < cnt && (int32_t)(sw[s] >> 32) == key) ? s : f;
  return f;
}

// NoDiskConflict (predicates.go:276-285 over isVolumeConflict :220-265): some volume of the pod
// is mounted on the node by a placed pod in a conflicting mode.
__device__ __forceinline__ uint32_t ksim_disk_conflict_body(const KsimVol& V, int32_t vclass, int64_t i) {
  const int32_t* vc = V.vc + 2 * (int64_t)(vclass - 1);
  const int32_t cnt = V.slot_count[i];
  if (cnt <= KSIM_VOL_REG) {
    uint64_t sw[KSIM_VOL_REG];
    ksim_vol_load_slots(V, i, cnt, sw);
    for (int32_t j = vc[0], e = vc[0] + vc[1]; j < e; ++j) {
      const ksim_vol_ref r = V.refs[j];
      if (!(r.flags & (KSIM_VOL_CONFLICT_ANY | KSIM_VOL_CONFLICT_RW))) continue;
      const int32_t s = ksim_vol_find_reg(sw, cnt, r.key);
      if (s < 0) continue;
      uint64_t w = 0;
#pragma unroll
      for (int t = 0; t < KSIM_VOL_REG; ++t) w = t == s ? sw[t] : w;
      const uint32_t rw = (uint32_t)(w & 0x7FFu), ro = (uint32_t)((w >> 11) & 0x7FFu);
      if ((r.flags & KSIM_VOL_CONFLICT_ANY) ? (rw + ro > 0) : (rw > 0)) return 1u << KSIM_R_DISK_CONFLICT;
    }
    return 0;
  }
  for (int32_t j = vc[0], e = vc[0] + vc[1]; j < e; ++j) {
    const ksim_vol_ref r = V.refs[j];
    if (!(r.flags & (KSIM_VOL_CONFLICT_ANY | KSIM_VOL_CONFLICT_RW))) continue;
    const int32_t s = ksim_vol_find(V, i, cnt, r.key);
    if (s < 0) continue;
    const uint64_t w = V.slots[(int64_t)s * V.n + i];
    const uint32_t rw = (uint32_t)(w & 0x7FFu), ro = (uint32_t)((w >> 11) & 0x7FFu);
    if ((r.flags & KSIM_VOL_CONFLICT_ANY) ? (rw + ro > 0) : (rw > 0)) return 1u << KSIM_R_DISK_CONFLICT;
  }
  return 0;
}
__device__ __noinline__ uint32_t ksim_disk_conflict(const KsimVol& V, int32_t vclass, int64_t i) { return ksim_disk_conflict_body(V, vclass, i); }

// MaxEBS / MaxGCEPD / MaxAzureDiskVolumeCount (predicates.go:415-456) for the filters in `which`,
// in that order: the node's distinct mounted keys the filter counts plus the pod's keys it counts
// that the node does not mount yet, against the filter's limit.
__device__ __forceinline__ uint32_t ksim_max_volumes_body(const KsimVol& V, int32_t vclass, int64_t i, uint32_t which) {
  const int32_t* vc = V.vc + 2 * (int64_t)(vclass - 1);
  const uint32_t want = V.vc_filter[vclass - 1] & which;
  if (!want) return 0;
  const int32_t cnt = V.slot_count[i];
  if (cnt <= KSIM_VOL_REG) {
    uint64_t sw[KSIM_VOL_REG];
    ksim_vol_load_slots(V, i, cnt, sw);
    uint32_t kf[KSIM_VOL_REG];  // the filters of the node's mounted keys, loaded together
#pragma unroll
    for (int s = 0; s < KSIM_VOL_REG; ++s) kf[s] = s < cnt ? V.key_filter[(int32_t)(sw[s] >> 32)] : 0u;
    for (int t = 0; t < 3; ++t) {
      const uint32_t f = 1u << t;
      if (!(want & f)) continue;
      int32_t have = 0;
#pragma unroll
      for (int s = 0; s < KSIM_VOL_REG; ++s) have += (kf[s] & f) ? 1 : 0;
      int32_t add = 0;
      for (int32_t j = vc[0], e = vc[0] + vc[1]; j < e; ++j) {
        const ksim_vol_ref r = V.refs[j];
        if ((r.flags & KSIM_VOL_NEW) && (V.key_filter[r.key] & f) && ksim_vol_find_reg(sw, cnt, r.key) < 0) ++add;
      }
      if (have + add > V.max_vols[t]) return 1u << KSIM_R_MAX_VOLUME_COUNT;
    }
    return 0;
  }
  for (int t = 0; t < 3; ++t) {
    const uint32_t f = 1u << t;
    if (!(want & f)) continue;
    int32_t have = 0;
    for (int32_t s = 0; s < cnt; ++s)
      if (V.key_filter[(int32_t)(V.slots[(int64_t)s * V.n + i] >> 32)] & f) ++have;
    int32_t add = 0;
    for (int32_t j = vc[0], e = vc[0] + vc[1]; j < e; ++j) {
      const ksim_vol_ref r = V.refs[j];
      if ((r.flags & KSIM_VOL_NEW) && (V.key_filter[r.key] & f) && ksim_vol_find(V, i, cnt, r.key) < 0) ++add;
    }
    if (have + add > V.max_vols[t]) return 1u << KSIM_R_MAX_VOLUME_COUNT;
  }
  return 0;
}
__device__ __noinline__ uint32_t ksim_max_volumes(const KsimVol& V, int32_t vclass, int64_t i, uint32_t which) { return ksim_max_volumes_body(V, vclass, i, which); }

__device__ __forceinline__ bool ksim_vol_zone_ok(const KsimVol& V, int32_t vclass, int32_t label_set) {
  if (!V.zone_ok) return true;
  return (V.zone_ok[(int64_t)(vclass - 1) * V.zone_words + (label_set >> 5)] >> (label_set & 31)) & 1u;
}

// NodeInfo.AddPod / RemovePod of a pod with volumes on node w (sign +1 / -1): each ref adds or
// takes one mount of its key (read-write, read-only or through a PVC).  Single thread; a full node
// or a saturated count sets err bit 1.
__device__ __forceinline__ void ksim_vol_commit_body(const KsimVol& V, const ksim_pod& P, int64_t w, int32_t sign,
                                             int32_t* err) {
  const int32_t* vc = V.vc + 2 * (int64_t)(P.vol_class - 1);
  for (int32_t j = vc[0], e = vc[0] + vc[1]; j < e; ++j) {
    const ksim_vol_ref r = V.refs[j];
    const int sh = (r.flags & KSIM_VOL_VIA_PVC) ? 22 : (r.flags & KSIM_VOL_READ_ONLY) ? 11 : 0;
    const uint64_t fmask = (sh == 22 ? 0x3FFull : 0x7FFull) << sh;
    const uint64_t one = 1ull << sh;
    const int32_t cnt = V.slot_count[w];
    const int32_t s = ksim_vol_find(V, w, cnt, r.key);
    uint64_t* slot = s >= 0 ? &V.slots[(int64_t)s * V.n + w] : nullptr;
    if (sign > 0) {
      if (slot) {
        if ((*slot & fmask) == fmask) atomicOr(err, 1);
        else *slot += one;
      } else if (cnt >= V.vol_slots) {
        atomicOr(err, 1);
      } else {
        V.slots[(int64_t)cnt * V.n + w] = ((uint64_t)(uint32_t)r.key << 32) | one;
        V.slot_count[w] = cnt + 1;
      }
    } else if (slot && (*slot & fmask)) {
      const uint64_t v = *slot - one;
      if ((v & 0xFFFFFFFFull) == 0) {  // no mount left: the slot goes (slot order is irrelevant)
        *slot = V.slots[(int64_t)(cnt - 1) * V.n + w];
        V.slots[(int64_t)(cnt - 1) * V.n + w] = 0;
        V.slot_count[w] = cnt - 1;
      } else {
        *slot = v;
      }
    }
  }
}
__device__ __noinline__ void ksim_vol_commit(const KsimVol& V, const ksim_pod& P, int64_t w, int32_t sign,
                                             int32_t* err) {
  ksim_vol_commit_body(V, P, w, sign, err);
}

// CheckServiceAffinity's labels from the lender (predicates.go:986-1011) for affinity class a on
// node i: the class's nodeSelector lacks the labels of svc_miss[a]; with cached pods matching its
// identity v (pair_all > 0), label l is constrained to the value their nodes share — unless none of
// them carries l (the pair at l's presence key is 0).  Disagreeing nodes (svc_conflict) make the
// reference's answer depend on the pod lister's order: err bit 128, the host refuses the run.
__device__ __forceinline__ uint32_t ksim_svc_lender(const KsimCtx& c, const KsimAff& A, int32_t a, int64_t i) {
  const int32_t v = A.svc_class[a];
  if (v < 0) return 0;
  const uint32_t miss = A.svc_miss[a];
  const ksim_svc_ident& S = A.svc[v];
  const int32_t total = A.cnt[A.pair_off[S.pair_all]];
  if (total == 0) return 0;  // no cached pod to lend labels
  if (A.svc_conflict[v] & miss) {
    atomicOr(c.err, 128);
    return 1u << KSIM_R_SERVICE_AFFINITY;
  }
  for (uint32_t mm = miss; mm; mm &= mm - 1) {
    const int l = __builtin_ctz(mm);
    if (A.cnt[A.pair_off[S.pair_present[l]]] == 0) continue;  // the lender lacks l: no constraint
    const int32_t pv = S.pair_value[l];
    const int32_t d = ksim_dom(A, A.pair_key[pv], i);
    if (d < 0 || A.cnt[A.pair_off[pv] + d] != total) return 1u << KSIM_R_SERVICE_AFFINITY;
  }
  return 0;
}

// Before the commit of pod P on node w adds its counts: the service-affinity identities whose
// selector P matches record the labels on which w disagrees with their earlier cached pods.
// Single thread.
__device__ __forceinline__ void ksim_svc_commit(const KsimAff& A, const ksim_pod& P, int64_t w) {
  if (!A.svc_class || P.aff_ident <= 0) return;
  for (int32_t e = A.svc_of_off[P.aff_ident - 1], end = A.svc_of_off[P.aff_ident]; e < end; ++e) {
    const int32_t v = A.svc_of[e];
    const ksim_svc_ident& S = A.svc[v];
    const int32_t total = A.cnt[A.pair_off[S.pair_all]];
    if (total == 0) continue;  // the first one: nothing to disagree with
    uint32_t bad = 0;
    for (int l = 0; l < A.n_svc_labels; ++l) {
      const int32_t pv = S.pair_value[l];
      const int32_t d = ksim_dom(A, A.pair_key[pv], w);
      const int32_t here = d >= 0 ? A.cnt[A.pair_off[pv] + d] : total - A.cnt[A.pair_off[S.pair_present[l]]];
      if (here != total) bad |= 1u << l;
    }
    if (bad) atomicOr(&A.svc_conflict[v], bad);
  }
}

// Reason mask of the first failing predicate in predicatesOrdering (predicates.go:129-138,
// core/generic_scheduler.go:467-528); 0 = fits.  IPA = false stops before MatchInterPodAffinity (the
// last key), for a kernel that evaluates it over its own count layout (ksim_pgen.hip).
// INL: the volume / affinity predicates inlined (the launch-form kernels) instead of called out of
// line (the persistent kernels, whose instruction-cache footprint they would grow)
template <class A, bool IPA = true, bool INL = false>
__device__ __forceinline__ uint32_t ksim_predicates_a(const KsimCtx& c, const ksim_pod& P, int64_t i, const KsimRow& r,
                                                      const A& a) {
  const uint32_t pr = c.preds;
  uint32_t m;
  if (pr & KSIM_P_CHECK_NODE_CONDITION) {
    m = r.fl & KSIM_COND_REASON_MASK;  // bit positions coincide with KSIM_R_*
    if (m) return m;
  }
  if ((pr & KSIM_P_CHECK_NODE_UNSCHEDULABLE) && (r.fl & KSIM_N_UNSCHEDULABLE)) return 1u << KSIM_R_UNSCHEDULABLE;
  if (pr & KSIM_P_GENERAL) {
    m = ksim_resources(c, P, i, r) | ksim_hostname(P, i);
    if (P.port_cnt) m |= ksim_hostports(c, P, i, a);
    m |= ksim_selector(P, i, a);
    if (m) return m;
  }
  if (pr & KSIM_P_HOSTNAME) {
    m = ksim_hostname(P, i);
    if (m) return m;
  }
  if ((pr & KSIM_P_HOST_PORTS) && P.port_cnt) {
    m = ksim_hostports(c, P, i, a);
    if (m) return m;
  }
  if (pr & KSIM_P_NODE_SELECTOR) {
    m = ksim_selector(P, i, a);
    if (m) return m;
  }
  if (pr & KSIM_P_RESOURCES) {
    m = ksim_resources(c, P, i, r);
    if (m) return m;
  }
  const bool vol = ksim_is_vol_pod(c, P);
  if ((pr & KSIM_P_DISK_CONFLICT) && vol) {
    m = INL ? ksim_disk_conflict_body(*c.vol, P.vol_class, i) : ksim_disk_conflict(*c.vol, P.vol_class, i);
    if (m) return m;
  }
  if ((pr & KSIM_P_TAINTS) && (P.flags & KSIM_POD_NEED_TAINTS)) {
    if (!a.taint_ok(P, i)) return 1u << KSIM_R_TAINTS;
  }
  if ((pr & KSIM_P_NOEXEC_TAINTS) && (P.flags & KSIM_POD_NEED_TAINTS)) {
    if (!a.noexec_ok(P, i)) return 1u << KSIM_R_TAINTS;
  }
  if ((pr & KSIM_P_LABEL_PRESENCE) && (r.fl & KSIM_N_LABEL_PRESENCE)) return 1u << KSIM_R_LABEL_PRESENCE;
  if ((pr & KSIM_P_SERVICE_AFFINITY) && (P.flags & KSIM_POD_NEED_SVC_AFFINITY) && c.svc_ok &&
      !ksim_bit(c.svc_ok, P.cls, c.lwords, c.label_set[i]))
    return 1u << KSIM_R_SERVICE_AFFINITY;
  if (INL && (pr & KSIM_P_SERVICE_AFFINITY) && c.aff && c.aff->svc_class && P.aff_class > 0) {
    m = ksim_svc_lender(c, *c.aff, P.aff_class - 1, i);
    if (m) return m;
  }
  if (vol) {
    const uint32_t which = ((pr & KSIM_P_MAX_EBS) ? KSIM_VOL_EBS : 0u) | ((pr & KSIM_P_MAX_GCE_PD) ? KSIM_VOL_GCE_PD : 0u) |
                           ((pr & KSIM_P_MAX_AZURE_DISK) ? KSIM_VOL_AZURE_DISK : 0u);
    if (which) {
      m = INL ? ksim_max_volumes_body(*c.vol, P.vol_class, i, which) : ksim_max_volumes(*c.vol, P.vol_class, i, which);
      if (m) return m;
    }
    if ((pr & KSIM_P_VOLUME_ZONE) && !ksim_vol_zone_ok(*c.vol, P.vol_class, c.label_set[i])) return 1u << KSIM_R_VOLUME_ZONE;
  }
  if ((pr & KSIM_P_MEM_PRESSURE) && (P.flags & KSIM_POD_BEST_EFFORT) && (r.fl & KSIM_N_MEM_PRESSURE))
    return 1u << KSIM_R_MEM_PRESSURE;
  if ((pr & KSIM_P_DISK_PRESSURE) && (r.fl & KSIM_N_DISK_PRESSURE)) return 1u << KSIM_R_DISK_PRESSURE;
  if (IPA && (pr & KSIM_P_INTERPOD_AFFINITY) && c.aff && (P.aff_ident > 0 || P.aff_class > 0))
    return INL ? ksim_interpod_pred_body(*c.aff, P, i) : ksim_interpod_pred(*c.aff, P, i);
  return 0;
}

__device__ __forceinline__ uint32_t ksim_predicates(const KsimCtx& c, const ksim_pod& P, int64_t i, const KsimRow& r) {
  return ksim_predicates_a<KsimGlobalAcc, true, true>(c, P, i, r, KsimGlobalAcc{c});
}

// Weighted sum of the map-type priorities (core/generic_scheduler.go:632-639); the reduce
// priorities are added per reduce class once their global maxima are known.
__device__ __forceinline__ int64_t ksim_map_score(const KsimCtx& c, const ksim_pod& P, const KsimRow& r) {
  if (c.no_prio) return 0;
  const int64_t rc = P.nz_cpu + r.zc;  // resource_allocation.go:58-59
  const int64_t rm = P.nz_mem + r.zm;
  uint64_t s = 0;  // Go int: wrapping
  if (c.w[KSIM_W_LEAST_REQUESTED])
    s += (uint64_t)c.w[KSIM_W_LEAST_REQUESTED] * (uint64_t)((ksim_least(rc, r.ac) + ksim_least(rm, r.am)) / 2);
  if (c.w[KSIM_W_MOST_REQUESTED])
    s += (uint64_t)c.w[KSIM_W_MOST_REQUESTED] * (uint64_t)((ksim_most(rc, r.ac) + ksim_most(rm, r.am)) / 2);
  if (c.w[KSIM_W_BALANCED])
    s += (uint64_t)c.w[KSIM_W_BALANCED] * (uint64_t)ksim_balanced(rc, r.ac, rm, r.am);
  return (int64_t)s;
}

template <class A>
__device__ __forceinline__ int ksim_rclass_a(const ksim_pod& P, int64_t i, int k1, int k2, const A& acc) {
  int a = 0, b = 0;
  if (k1 > 1) a = acc.tt_class(P, i);
  if (k2 > 1) b = acc.na_class(P, i);
  return a * k2 + b;
}

__device__ __forceinline__ int ksim_rclass(const KsimCtx& c, const ksim_pod& P, int64_t i, int k1, int k2) {
  return ksim_rclass_a(P, i, k1, k2, KsimGlobalAcc{c});
}

// NormalizeReduce (priorities/reduce.go:29-64) applied to one class value.
__device__ __forceinline__ int64_t ksim_norm(int64_t v, int64_t mx, bool reverse) {
  if (mx == 0) return reverse ? 10 : v;
  int64_t s;
  if (v >= 0 && v < (int64_t(1) << 20) && mx > 0 && mx < (int64_t(1) << 24)) {
    // the common case (taint counts, preference weights): both operands exact in float32 and
    // the quotient <= 10 for v <= mx, so an approximate reciprocal is within one of the
    // truncated quotient and one integer correction makes it exact
    const int32_t x = 10 * (int32_t)v, m = (int32_t)mx;
    int32_t q = (int32_t)((float)x * __builtin_amdgcn_rcpf((float)m));
    if (q * m > x) q -= 1;
    else if ((q + 1) * m <= x) q += 1;
    s = q;
  } else if (v >= 0 && v < (int64_t(1) << 40) && mx > 0 && mx < (int64_t(1) << 40)) {
    // map values are small: a correctly rounded float64 quotient plus one integer correction
    // is Go's truncating int64 division (ksim_mul10_div), without the emulated 64-bit divide
    const int64_t x = 10 * v;
    s = (int64_t)((double)x / (double)mx);
    if (s * mx > x) s -= 1;
    else if ((s + 1) * mx <= x) s += 1;
  } else {
    s = ksim_mul10_div_slow(v, mx);
  }
  return reverse ? 10 - s : s;
}

// Commit pod P to node w: NodeInfo.AddPod (node_info.go:318-341) + HostPortInfo.Add
// (utils.go:45-60).  Single thread.
__device__ __forceinline__ void ksim_commit(const KsimCtx& c, const ksim_pod& P, int64_t w) {
  c.req_cpu[w] += P.add_cpu;
  c.req_mem[w] += P.add_mem;
  const int64_t g = c.req_gpu[w] + P.add_gpu;
  const int64_t e = c.req_eph[w] + P.add_eph;
  c.req_gpu[w] = g;
  c.req_eph[w] = e;
  c.nz_cpu[w] += P.nz_cpu;
  c.nz_mem[w] += P.nz_mem;
  c.pod_count[w] += 1;
  uint32_t fl = c.flags[w] & ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
  if (c.alloc_gpu[w] < g) fl |= KSIM_N_GPU_OVER;
  if (c.alloc_eph[w] < e) fl |= KSIM_N_EPH_OVER;
  c.flags[w] = fl;
  for (int32_t s = 0; s < P.scalar_cnt; ++s) {
    const ksim_scalar_req q = ksim_pod_scalar(c, P, s);
    c.req_scalar[(int64_t)q.col * c.n + w] += q.add;
  }
  for (int32_t k = 0; k < P.port_cnt; ++k) {
    const uint64_t key = ksim_pod_port(c, P, k);
    int32_t cnt = c.port_count[w];
    bool dup = false;
    for (int32_t s = 0; s < cnt; ++s)
      if (c.ports[(int64_t)s * c.n + w] == key) { dup = true; break; }
    if (dup) continue;
    if (cnt >= c.port_slots) { atomicOr(c.err, 1); continue; }
    c.ports[(int64_t)cnt * c.n + w] = key;
    c.port_count[w] = cnt + 1;
  }
}

// Status of a committed row for the fast kernels' float64 arithmetic (ksim_pfast.hip,
// ksim_tree.hip): bit 0 set when a cpu / memory quantity left [0, 2^48).
__device__ __forceinline__ int32_t ksim_row_status(const KsimCtx& c, int64_t w) {
  const int64_t lim = int64_t(1) << 48;
  const int64_t a = c.req_cpu[w], b = c.req_mem[w], d = c.nz_cpu[w], e = c.nz_mem[w];
  return (a < 0 || a >= lim || b < 0 || b >= lim || d < 0 || d >= lim || e < 0 || e >= lim) ? 1 : 0;
}

// ksim_commit by one wave (lane = 0..63, every lane calls): lane 0 updates the row's columns and
// returns ksim_row_status of the committed values (bit 0), and for a pod with host ports bit 1 and
// the row's port count after the commit in bits 8.. (the host keeps its port-slot bound exact);
// the host-port dedup reads the row's port slots in parallel (one lane a slot).
__device__ __forceinline__ int32_t ksim_commit_wave(const KsimCtx& c, const ksim_pod& P, int64_t w, int lane) {
  int32_t st = 0;
  if (lane == 0) {
    const int64_t rc = c.req_cpu[w] + P.add_cpu, rm = c.req_mem[w] + P.add_mem;
    const int64_t g = c.req_gpu[w] + P.add_gpu, e = c.req_eph[w] + P.add_eph;
    const int64_t zc = c.nz_cpu[w] + P.nz_cpu, zm = c.nz_mem[w] + P.nz_mem;
    const int32_t pc = c.pod_count[w] + 1;
    uint32_t fl = c.flags[w] & ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
    if (c.alloc_gpu[w] < g) fl |= KSIM_N_GPU_OVER;
    if (c.alloc_eph[w] < e) fl |= KSIM_N_EPH_OVER;
    c.req_cpu[w] = rc; c.req_mem[w] = rm; c.req_gpu[w] = g; c.req_eph[w] = e;
    c.nz_cpu[w] = zc; c.nz_mem[w] = zm; c.pod_count[w] = pc; c.flags[w] = fl;
    for (int32_t s = 0; s < P.scalar_cnt; ++s) {
      const ksim_scalar_req q = ksim_pod_scalar(c, P, s);
      c.req_scalar[(int64_t)q.col * c.n + w] += q.add;
    }
    const int64_t lim = int64_t(1) << 48;
    st = (rc < 0 || rc >= lim || rm < 0 || rm >= lim || zc < 0 || zc >= lim || zm < 0 || zm >= lim) ? 1 : 0;
  }
  if (P.port_cnt == 0) return st;
  if (c.port_slots > 64) {  // wider than a wave: the serial form
    if (lane == 0) {
      int32_t cnt = c.port_count[w];
      for (int32_t k = 0; k < P.port_cnt; ++k) {
        const uint64_t key = ksim_pod_port(c, P, k);
        bool dup = false;
        for (int32_t s = 0; s < cnt; ++s)
          if (c.ports[(int64_t)s * c.n + w] == key) { dup = true; break; }
        if (dup) continue;
        if (cnt >= c.port_slots) { atomicOr(c.err, 1); continue; }
        c.ports[(int64_t)cnt * c.n + w] = key;
        c.port_count[w] = ++cnt;
      }
      st |= 2 | (cnt << 8);
    }
    return st;
  }
  const int32_t cnt0 = c.port_count[w];
  uint64_t mine = lane < cnt0 ? c.ports[(int64_t)lane * c.n + w] : 0ull;
  int32_t cnt = cnt0;
  for (int32_t k = 0; k < P.port_cnt; ++k) {  // uniform: the pod's keys in order
    const uint64_t key = ksim_pod_port(c, P, k);
    if (__ballot(lane < cnt && mine == key)) continue;
    if (cnt >= c.port_slots) {
      if (lane == 0) atomicOr(c.err, 1);
      continue;
    }
    if (lane == cnt) mine = key;
    if (lane == 0) c.ports[(int64_t)cnt * c.n + w] = key;
    ++cnt;
  }
  if (lane == 0 && cnt != cnt0) c.port_count[w] = cnt;
  return st | 2 | (cnt << 8);
}

// Undo a commit of pod P on row w exactly (a tentative commit the host did not confirm): the
// arithmetic inverse of ksim_commit_wave — quantities back, pod count back, the row's port count
// and flags as they were before (its new keys were appended past cnt0).  Single thread.
__device__ __forceinline__ void ksim_undo_commit(const KsimCtx& c, const KsimTentRec& t) {
  const int64_t w = t.node;
  const ksim_pod& P = t.P;
  c.req_cpu[w] -= P.add_cpu;
  c.req_mem[w] -= P.add_mem;
  c.req_gpu[w] -= P.add_gpu;
  c.req_eph[w] -= P.add_eph;
  c.nz_cpu[w] -= P.nz_cpu;
  c.nz_mem[w] -= P.nz_mem;
  c.pod_count[w] -= 1;
  c.flags[w] = t.fl0;
  for (int32_t s = 0; s < P.scalar_cnt; ++s) c.req_scalar[(int64_t)t.sc[s].col * c.n + w] -= t.sc[s].add;
  if (P.port_cnt) c.port_count[w] = t.cnt0;
}

// Remove pod P from node w: NodeInfo.RemovePod (node_info.go:343-390) — the containers-only
// requests and non-zero requests are subtracted, the pod count drops by one and the pod's
// (ip, protocol, port) keys leave the node's HostPortInfo (HostPortInfo.Remove, utils.go:63-79,
// set semantics: the key goes even if another pod added it too).  Single thread.
__device__ __forceinline__ void ksim_uncommit(const KsimCtx& c, const ksim_pod& P, int64_t w) {
  c.req_cpu[w] -= P.add_cpu;
  c.req_mem[w] -= P.add_mem;
  const int64_t g = c.req_gpu[w] - P.add_gpu;
  const int64_t e = c.req_eph[w] - P.add_eph;
  c.req_gpu[w] = g;
  c.req_eph[w] = e;
  c.nz_cpu[w] -= P.nz_cpu;
  c.nz_mem[w] -= P.nz_mem;
  c.pod_count[w] -= 1;
  uint32_t fl = c.flags[w] & ~(KSIM_N_GPU_OVER | KSIM_N_EPH_OVER);
  if (c.alloc_gpu[w] < g) fl |= KSIM_N_GPU_OVER;
  if (c.alloc_eph[w] < e) fl |= KSIM_N_EPH_OVER;
  c.flags[w] = fl;
  for (int32_t s = 0; s < P.scalar_cnt; ++s) {
    const ksim_scalar_req q = ksim_pod_scalar(c, P, s);
    c.req_scalar[(int64_t)q.col * c.n + w] -= q.add;
  }
  for (int32_t k = 0; k < P.port_cnt; ++k) {
    const uint64_t key = ksim_pod_port(c, P, k);
    const int32_t cnt = c.port_count[w];
    for (int32_t s = 0; s < cnt; ++s) {
      if (c.ports[(int64_t)s * c.n + w] != key) continue;
      c.ports[(int64_t)s * c.n + w] = c.ports[(int64_t)(cnt - 1) * c.n + w];  // slot order is irrelevant
      c.ports[(int64_t)(cnt - 1) * c.n + w] = 0;
      c.port_count[w] = cnt - 1;
      break;
    }
  }
}
