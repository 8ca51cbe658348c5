// ksim_handle.h — private host-side state of a ksim_handle, shared by the runtime
// translation units (ksim_runtime.cpp: load / schedule / sweep / shard; ksim_cache.cpp: the
// per-pod drop-in entry points and the scheduler-cache event mirror).  Not part of the C-ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <array>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "ksim_common.h"
#include "ksim_pgen.h"
#include "ksim_sweep.h"
#include "ksim_tree.h"
#include "ksim_f64.h"

// ---- kernel launchers (the .hip translation units) ----
extern "C" hipError_t ksim_launch_scan(const KsimCtx* c, int npt, int collect, int grid, hipStream_t s);
extern "C" hipError_t ksim_launch_eval(const KsimCtx* c, int64_t pod, uint8_t* fit, uint32_t* reasons, int64_t* score,
                                       uint8_t* rcls, hipStream_t s);
extern "C" int ksim_scan_coresident(int npt, int collect, int grid);
extern "C" int ksim_one_npt(int64_t n);
extern "C" hipError_t ksim_launch_one(const KsimCtx* c, int npt, hipStream_t s);
extern "C" int ksim_pick_coresident(int npt, int grid);
extern "C" hipError_t ksim_launch_pick(const KsimCtx* c, int npt, int grid, int aux, hipStream_t s);
extern "C" int ksim_serve_coresident(int npt, int grid);
extern "C" hipError_t ksim_launch_serve(const KsimCtx* c, const KsimServeArgs* a, int npt, int grid, int aux, hipStream_t s);
extern "C" hipError_t ksim_launch_ipa_pass(const KsimCtx* c, int npt, int grid, hipStream_t s);
extern "C" hipError_t ksim_launch_assume(const KsimCtx* c, int64_t pod, int64_t node, int32_t* status, hipStream_t s);
extern "C" hipError_t ksim_launch_persistent(const KsimCtx* c, const KsimCtx* cdev, uint64_t* granules, int grid,
                                             int lds_rows, hipStream_t s);
extern "C" int ksim_persistent_config(int64_t n, int* grid, int* lds_rows);
extern "C" size_t ksim_persistent_granule_bytes(int grid);
extern "C" hipError_t ksim_sweep_prepare(const int64_t* ac, const int64_t* am, int64_t n, double* dac, double* dam,
                                         double* yc, double* ym, hipStream_t st);
extern "C" hipError_t ksim_sweep_launch(const int64_t* rc0, const int64_t* rm0, const int64_t* zc0, const int64_t* zm0,
                                        const int32_t* c0, const ksim_pod* pods, void* fpods, const SwArgs* args,
                                        int32_t n_scen, hipEvent_t ev0, hipEvent_t ev1, hipStream_t st);
extern "C" int ksim_pfast_config(int64_t n, int max_grid, int stream, int* grid, int* lds_rows);
extern "C" hipError_t ksim_pstream_prepare(const KsimCtx* c, double* mirror, hipStream_t s);
extern "C" size_t ksim_pfast_granule_bytes(void);
extern "C" size_t ksim_shard_xchg_bytes(void);
extern "C" size_t ksim_shard_lx_offset(void);
extern "C" size_t ksim_pfast_cache_bytes(int lds_rows, int ncls);
extern "C" hipError_t ksim_launch_pfast(const KsimCtx* c, uint64_t* granules, int grid, int lds_rows, double* mirror,
                                        const KsimShard* sh, const int32_t* tcls, const KsimTreeClass* tclass, int ncls,
                                        hipStream_t s);
extern "C" hipError_t ksim_tree_build(const KsimCtx* c, const KsimTreeGeo* g, const KsimTreeClass* cls,
                                      const int32_t* tcls, int32_t* leaves, uint64_t* levels, int32_t* fitc,
                                      double* ty, const KsimTreeSweep* sw, hipStream_t s);
extern "C" hipError_t ksim_tree_sweep_init(const KsimCtx* c, const KsimTreeSweep* sw, hipStream_t s);
extern "C" hipError_t ksim_tree_launch(const KsimCtx* c, const KsimTreeGeo* g, const KsimTreeClass* cls,
                                       const int32_t* tcls, int32_t* leaves, uint64_t* levels, int32_t* fitc,
                                       double* ty, const KsimTreeSweep* sw, hipStream_t s);
// scheduler-cache kernels (ksim_cache.hip)
struct KsimRelayout;
extern "C" hipError_t ksim_launch_relayout(const KsimRelayout* r, hipStream_t s);
extern "C" hipError_t ksim_launch_set_row(const KsimCtx* c, int64_t node, const uint64_t* pack, int32_t full,
                                          hipStream_t s);
extern "C" hipError_t ksim_launch_release(const KsimCtx* c, int64_t pod, int64_t node, hipStream_t s);
extern "C" hipError_t ksim_launch_undo(const KsimCtx* c, const KsimTentRec* t, hipStream_t s);
extern "C" hipError_t ksim_launch_remap_hosts(ksim_pod* pods, int64_t n_pods, int64_t idx, int32_t op, hipStream_t s);
extern "C" hipError_t ksim_launch_pod_k(ksim_pod* pods, int64_t n_pods, const KsimCtx* c, hipStream_t s);
extern "C" hipError_t ksim_launch_port_max(const int32_t* port_count, int64_t n, int32_t* out, hipStream_t s);

struct DevBuf {
  void* p = nullptr;
  size_t bytes = 0;
};

// Per-pod staging area of the drop-in entry points (ksim_schedule_one, ksim_pod_add/remove): one
// block of pinned host memory mapped into the device's address space — {cursor, result block, pod,
// ports, scalars} — that the kernels read the pod from and write the result to directly, so a call
// is one launch and one stream sync, with no copy either way.
// (the result block layout KSIM_RES_* is in ksim_common.h: the kernels write it)

// The small volume tables' segments in vol_small (ksim_volumes.cpp): capacities, the loaded ref
// count and byte offsets, so a grow within the capacities writes only the new entries.
struct VolSeg {
  bool valid = false;
  int64_t cap_keys = 0, cap_vclass = 0, cap_refs = 0;
  int32_t n_refs = 0;
  size_t o_kf = 0, o_vc = 0, o_vf = 0, o_refs = 0, o_zo = 0;
};

struct ksim_handle {
  int device = 0;
  // the handle's one stream: every launch and copy goes through ksim_stream(h), which first stops
  // the resident per-pod kernel when it is running (so nothing ever queues behind it)
  hipStream_t stream_raw = nullptr;
  hipEvent_t ev0 = nullptr, ev1 = nullptr;
  ksim_config cfg{};
  std::string err;
  std::vector<DevBuf> bufs;
  KsimCtx ctx{};
  bool have_nodes = false, have_classes = false, have_pods = false;
  bool any_wide = false;  // some pod class has more than KSIM_MAX_RCLASS reduce classes
  int64_t n_pods = 0, pod_cap = 0;
  int64_t n_port_keys = 0, port_key_cap = 0;     // pod-port array (queue)
  int64_t n_scalar_reqs = 0, scalar_req_cap = 0; // pod-scalar array (queue)
  ksim_pod* d_pods = nullptr;                    // non-const views of the queue arrays in ctx
  uint64_t* d_pod_ports = nullptr;
  ksim_scalar_req* d_pod_scalars = nullptr;
  int32_t n_classes = 0;
  int32_t n_label_sets = 0, n_taint_sets = 0;   // of the loaded class tables
  int32_t max_label_set = -1, max_taint_set = -1;  // largest ids the node table uses
  std::vector<void*> class_bufs;                 // class-table buffers (replaced when they grow)
  // class tables at capacity strides + their pinned host mirror (ksim_load_classes)
  struct {
    int64_t cap_c = 0, cap_l = 0, cap_t = 0;  // capacities (the device strides)
    int64_t c = 0, l = 0, t = 0;              // loaded
    int64_t w = 0;                            // value row width (ksim_class_tables.val_width)
    bool has_na = false, has_sv = false;
    char* mirror = nullptr;
    int64_t loads = 0, in_place = 0;          // reloads, and those written beside a running resident kernel
  } cls;
  hipStream_t side_stream = nullptr;             // table writes beside the resident per-pod kernel
  // launch-mode graph
  hipGraphExec_t gexec = nullptr;
  hipGraph_t graph = nullptr;
  int g_batch = 0, g_npt = 0, g_collect = -1, g_ipa = -1, part_cap = 0;
  uint64_t* granules = nullptr;
  KsimCtx* ctx_dev = nullptr;  // device copy of ctx for non-inlined device functions
  size_t gran_bytes = 0;
  int64_t g_first = -1, g_end = -1;
  // host-side copies needed for validation
  std::vector<int32_t> h_n_tt, h_n_na;
  // per queued pod: class and "resource-only apart from its reduce classes" (ksim_is_fast_pod)
  std::vector<int32_t> q_cls;
  std::vector<uint8_t> q_base;
  // fast_pre[i] = resource-only pods among the first i of the queue (ksim_is_fast_pod)
  std::vector<int64_t> fast_pre;
  // the fast kernel computes in float64: every node cpu / memory quantity below 2^48 at load
  // (pods: checked per pod in fast_pre); cleared for good once a commit reaches 2^48
  bool pfast_off = false;
  std::vector<int64_t> pod_qmax;  // largest cpu / memory quantity of each pod (sweep bound)
  // scenario sweep: static float64 columns (once) and per-call scratch (grown on demand)
  double *sw_dac = nullptr, *sw_dam = nullptr, *sw_yc = nullptr, *sw_ym = nullptr;
  void* sw_scratch = nullptr;
  size_t sw_scratch_bytes = 0;
  // node-sharded mode (ksim_shard_*): world == 1 is the ordinary single-device mode
  KsimShard shard{0, 1, 0, 0, nullptr, {}, 0};
  void* ipc_mapped[KSIM_MAX_RANKS] = {};  // peers' exchange buffers opened through IPC
  int max_grid = 0;                        // workgroups per launch (0 = one per CU)
  double* mirror = nullptr;                // streaming fast kernel: float64 image [6][n]
  int64_t mirror_n = 0;
  // tree mode (ksim_tree.hip): tree class of every resource-only pod (-1 otherwise), the class
  // inputs, the geometry and the device trees; tree_valid = the trees describe the current
  // node table (any other commit path clears it)
  int32_t n_tcls = 0;                      // -1: more classes than the tree supports
  bool last_pfast_cache = false;           // the last fast-kernel call took the cached form
  uint64_t* pick_words = nullptr;          // the per-pod pick kernel's exchange records
  uint32_t pick_tag = 0;
  int pick_grid = -1, pick_npt = -1;
  bool pick_ok = false;
  bool pick_clear = false;                 // the record buffers must be zeroed before the next call (new geometry)
  bool serve_fits = false;                 // the resident kernel's grid for (pick_npt, pick_grid) is co-resident
  // the resident per-pod service (ksim_serve_kernel, ksim_cache.cpp): mailbox, the context and
  // geometry it was launched with, per-block pod staging, the last message posted.  serve_live is
  // read without the device gate by ksim_stream (another handle's exclusive section may clear it)
  std::atomic<bool> serve_live{false};
  bool serve_off = false;                  // KSIM_SERVE=0, or a failure: per-pod launches only
  KsimServeBox* serve_box = nullptr;       // coherent host memory ...
  KsimServeBox* serve_box_dev = nullptr;   // ... as the device addresses it
  uint64_t* serve_state = nullptr;         // device: the grid's idle vote (KSIM_SERVE_ST_*)
  KsimCtx serve_base{};                    // h->ctx when the kernel was launched
  int serve_npt = 0, serve_grid = 0;
  bool serve_aux = false;  // the resident kernel's instantiation reads the auxiliary priority
  uint64_t serve_seq = 0;
  uint32_t serve_launch_id = 0;
  bool serve_shared = false;               // the last message committed state other blocks read
  char* serve_stage = nullptr;             // device: [grid] pods, [grid][KSIM_ONE_PORTS] ports, [grid][KSIM_MAX_SCALAR] scalars
  // launches, messages, stops, relaunches after the grid left by its idle vote, messages served by
  // such a relaunch (the grid left before taking them)
  int64_t serve_stats[5] = {0, 0, 0, 0, 0};
  // lastNodeIndex as the host last saw it in a resident kernel's answer, while nothing else can
  // have changed the device word (cleared by ksim_stream, kept across counter-neutral calls): the
  // next launch starts from it, and each answer is checked against it (selectHost bumps it by one
  // exactly when two or more nodes fit, generic_scheduler.go:183-198)
  uint64_t ctr_host = 0;
  bool ctr_known = false;
  // the adapter's SCHEDULE_ONLY + AssumePod pattern in one message: a tentative commit (the resident
  // kernel commits a SCHEDULE_ONLY pod and keeps a record; a ksim_pod_add naming the same pod and
  // node confirms it without a message, anything else undoes it first — ksim_cache.cpp)
  struct {
    bool live = false;            // the rows hold a commit the host has not decided on
    bool undo_inflight = false;   // decided "undo", carried by messages, not yet acknowledged
    uint32_t launch = 0;          // the resident launch that holds the record
    int32_t act = 0;              // what messages tell the kernel about rec.seq (KSIM_TENT_*)
    KsimTentRec rec{};            // (ports: rec.P.port_cnt of them in ports)
    uint64_t ports[KSIM_ONE_PORTS] = {};
    int32_t res[KSIM_RES_WORDS] = {};  // its answer (status / error for the confirming assume)
  } tent;
  int64_t tent_stats[4] = {0, 0, 0, 0};  // tentative commits, undone, undone by a launch, confirmed
  int32_t* tcls = nullptr;
  int64_t tcls_cap = 0;
  KsimTreeClass* tclass = nullptr;
  std::map<std::array<int64_t, 5>, int32_t> tkeys;
  std::vector<KsimTreeClass> tclass_h;
  bool tree_planned = false, tree_ok = false, tree_valid = false;
  KsimTreeGeo geo{};
  int32_t* t_leaves = nullptr;
  uint64_t* t_levels = nullptr;
  int32_t* t_fit = nullptr;
  double* t_y = nullptr;
  void* swt_scratch = nullptr;  // tree sweep: per-scenario columns, trees, counters, outputs
  size_t swt_bytes = 0;
  // per-pod drop-in staging (ksim_cache.cpp)
  char* stg_dev = nullptr;      // the mapped staging block as the device addresses it
  char* stg_host = nullptr;     // pinned host memory: [int64 cursor][result block][ksim_pod][ports][scalars]
  size_t stg_cap = 0;
  int32_t* res_dev = nullptr;   // result block (KSIM_RES_*), device view
  int32_t* res_host = nullptr;  // the same words, host view
  int64_t port_bound = 0;       // upper bound of max(port_count) over the nodes
  // inter-pod affinity (ksim_load_affinity): the device tables, their sizes for validation, and
  // per queued pod its identity / class (an affinity pod takes the launch-mode kernels)
  bool have_aff = false;
  bool aff_stale = false;       // a node event changed the table the domains describe
  int32_t aff_n_ident = 0, aff_n_aclass = 0;
  KsimAff* aff_dev = nullptr;
  KsimAff aff_h{};              // host copy of the device descriptor (pass-A scratch pointers)
  // general persistent kernel (ksim_pgen.hip): per identity / affinity class "its counts live in a
  // shared topology domain" flags, the tables' sizes, and the row-form count arrays + exchange buffer
  uint8_t* aff_ident_shared = nullptr;
  uint8_t* aff_aclass_shared = nullptr;
  int32_t aff_n_pair = 0, aff_n_carry = 0, aff_n_zone = 0, aff_n_keys = 0;
  // identity lists for the pod-context records (CSR, device): carried anti / priority terms the
  // identity matches, counted pairs it matches as (pair, key); and the longest list of each kind
  // over identities / affinity classes (the record-size bound)
  int32_t *pg_id_anti_off = nullptr, *pg_id_anti = nullptr, *pg_id_prio_off = nullptr, *pg_id_prio = nullptr;
  int32_t *pg_id_mp_off = nullptr, *pg_id_mp = nullptr;
  int32_t pg_max_anti = 0, pg_max_prio = 0, pg_max_mp = 0, pg_max_req = 0, pg_max_pref = 0, pg_max_car = 0;
  int32_t vol_max_ref = 0;                 // longest volume class
  int32_t q_max_port = 0, q_max_scal = 0;  // most host ports / scalar requests of a queued pod
  uint64_t* pg_gran = nullptr;
  char* pg_rec = nullptr;                  // pod-context records of the current call
  size_t pg_rec_bytes = 0;
  bool fuse_off = false;        // a fused pass-A barrier timed out once: pass A as its own launch
  int one_fuse_grid = -1;       // ksim_schedule_one: the grid whose co-residency was checked ...
  bool one_fuse_ok = false;     // ... and whether the fused pass A may run on it
  bool pgen_off = false;        // a general persistent kernel ran out of a spin bound once: the launch form
  std::vector<void*> aff_bufs;
  std::vector<int32_t> q_ident, q_aclass;
  std::vector<int64_t> aff_pre;  // aff_pre[i] = affinity pods among the first i queued
  // volumes (ksim_load_volumes): the device tables, the host copy of their descriptor (slot
  // pointers for ksim_read_volumes) and per queued pod its volume class (a volume pod takes the
  // launch-mode kernels)
  bool have_vol = false;
  bool vol_stale = false;       // a node event changed the table the slots describe
  int32_t vol_n_class = 0;
  int32_t vol_n_keys = 0;
  KsimVol vol_h{};
  KsimVol* vol_dev = nullptr;
  std::vector<void*> vol_bufs;  // the mounts (slots, slot_count) of the current tables
  // the small volume tables (KsimVol at offset 0, then key / class / ref / zone arrays) in one
  // persistent device buffer grown geometrically, so that ksim_grow_volumes is one upload
  char* vol_small = nullptr;
  size_t vol_small_cap = 0;
  std::vector<char> vol_small_host;
  int64_t vol_in_place = 0;      // grows written beside a running resident per-pod kernel
  VolSeg vol_seg;
  std::vector<int32_t> q_vclass;
  std::vector<int64_t> vol_pre;  // vol_pre[i] = volume / service-affinity pods among the first i queued
};

int ksim_fail(ksim_handle* h, int code, const char* fmt, ...);
// Stop the resident per-pod kernel (an exit message and a stream drain); KSIM_OK when none runs.
int ksim_serve_stop(ksim_handle* h);
// The handle leaves the device gate's list of running resident kernels (ksim_destroy).
void ksim_serve_forget(ksim_handle* h);
// Settle a tentative commit before any other use of the handle's state: undo it (ksim_cache.cpp).
int ksim_tent_undo(ksim_handle* h);
inline hipStream_t ksim_stream(ksim_handle* h) {
  if (h->tent.live) (void)ksim_tent_undo(h);  // (the stop below carries the undo to the kernel)
  if (h->serve_live.load(std::memory_order_acquire)) (void)ksim_serve_stop(h);
  h->ctr_known = false;  // (the stream's next use may change lastNodeIndex)
  return h->stream_raw;
}
// A call that cannot change lastNodeIndex (cache events, reads): the host's copy survives its
// stream uses.
struct KsimCtrKeep {
  ksim_handle* h;
  bool known;
  uint64_t v;
  explicit KsimCtrKeep(ksim_handle* hh) : h(hh), known(hh && hh->ctr_known), v(hh ? hh->ctr_host : 0) {}
  ~KsimCtrKeep() {
    if (h && known) { h->ctr_known = true; h->ctr_host = v; }
  }
};
// The device gate (ksim_cache.cpp).  A kernel whose blocks wait on each other (the persistent
// batch kernels, the per-pod pick kernel, the fused pass-A scan, the node-sharded kernels) must
// not share the device with another handle's resident per-pod kernel, which holds CUs between
// calls: such launches run with the gate taken "exclusive", which waits for every resident
// section to end, holds new ones back and stops every other handle's resident kernel on the
// device; the resident kernels' calls take it "shared".  Exclusive holders do not exclude each
// other (node-sharded ranks on one device).  Nested holds by one thread are free.
struct KsimGate {
  int dev = -1;
  int mode = 0;  // 0: not taken here, 1 shared, 2 exclusive
  KsimGate(ksim_handle* h, bool exclusive);
  ~KsimGate();
  KsimGate(const KsimGate&) = delete;
  KsimGate& operator=(const KsimGate&) = delete;
};

#define HIPCHK(h, x)                                                                              \
  do {                                                                                            \
    hipError_t e_ = (x);                                                                          \
    if (e_ != hipSuccess) return ksim_fail((h), KSIM_E_DEVICE, "%s: %s", #x, hipGetErrorString(e_)); \
  } while (0)

template <class T>
static int dev_alloc(ksim_handle* h, T** out, size_t count) {
  *out = nullptr;
  size_t bytes = std::max<size_t>(count * sizeof(T), 16);
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, bytes);
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_NOMEM, "hipMalloc(%zu): %s", bytes, hipGetErrorString(e));
  h->bufs.push_back({p, bytes});
  *out = reinterpret_cast<T*>(p);
  return KSIM_OK;
}

template <class T>
static int dev_upload(ksim_handle* h, T** out, const T* src, size_t count, bool zero_if_null = true) {
  int rc = dev_alloc(h, out, count);
  if (rc) return rc;
  if (src && count) {
    HIPCHK(h, hipMemcpyAsync(*out, src, count * sizeof(T), hipMemcpyHostToDevice, ksim_stream(h)));
  } else if (zero_if_null && count) {
    HIPCHK(h, hipMemsetAsync(*out, 0, count * sizeof(T), ksim_stream(h)));
  }
  return KSIM_OK;
}

// Free one buffer of the handle (the stream is drained first: hipFree must not race queued work).
static inline void dev_free(ksim_handle* h, const void* p) {
  if (!p) return;
  (void)hipStreamSynchronize(ksim_stream(h));
  (void)hipFree(const_cast<void*>(p));
  h->bufs.erase(std::remove_if(h->bufs.begin(), h->bufs.end(), [p](const DevBuf& b) { return b.p == p; }),
                h->bufs.end());
}

// Grow a device array to new_cap elements keeping the first `keep` elements.
template <class T>
static int dev_grow(ksim_handle* h, T** p, size_t keep, size_t new_cap) {
  T* q = nullptr;
  int rc = dev_alloc(h, &q, new_cap);
  if (rc) return rc;
  if (*p && keep) HIPCHK(h, hipMemcpyAsync(q, *p, keep * sizeof(T), hipMemcpyDeviceToDevice, ksim_stream(h)));
  dev_free(h, *p);
  *p = q;
  return KSIM_OK;
}

// ---- runtime internals shared across translation units (ksim_runtime.cpp) ----
// Append pods to the queue (first call: the initial load).  Validates, grows the device
// arrays, extends the per-pod host bookkeeping (fast-kernel eligibility, tree classes).
int ksim_rt_append(ksim_handle* h, const ksim_pod* pods, int64_t n_pods, const uint64_t* ports, int64_t n_ports,
                   const ksim_scalar_req* scalars, int64_t n_scalars);
// Recompute fast_pre from q_cls / q_base after the class tables changed.
void ksim_rt_recompute_fast(ksim_handle* h);
// Everything derived from the node table's size, pointers or static columns is stale
// (launch graph, tree geometry, sweep statics, streaming mirror).
void ksim_rt_invalidate_layout(ksim_handle* h);
// Validate one pod descriptor against the loaded tables (ports / scalars relative to the
// passed arrays).
int ksim_rt_check_pod(ksim_handle* h, const ksim_pod& p, int64_t n_ports, int64_t n_scalars,
                      const ksim_scalar_req* scalars, const char* where);
int ksim_rt_ensure_partials(ksim_handle* h, int grid);
// Affinity pods among queued pods [first, first+count).
int64_t ksim_rt_aff_count(const ksim_handle* h, int64_t first, int64_t count);
// Pods among [first, first+count) that only the launch-mode kernels schedule (affinity, volumes).
int64_t ksim_rt_launch_only_count(const ksim_handle* h, int64_t first, int64_t count);
// KSIM_E_STATE when the affinity or volume tables are stale (a node event since they were loaded).
int ksim_rt_check_aff(ksim_handle* h, const char* where);
int ksim_rt_pick_npt(int64_t n);
// The loaded affinity tables carry an auxiliary priority (ksim_affinity_tables.aux_*): only the
// launch-form kernels read it, so every pod of such a handle takes that form.
inline bool ksim_rt_aux_on(const ksim_handle* h) {
  return h->have_aff && h->aff_h.aux_pair != nullptr && h->aff_h.aux_w != 0 && !h->ctx.no_prio;
}
// The service-affinity lender check (ksim_affinity_tables.svc_*).
inline bool ksim_rt_svc_lender_on(const ksim_handle* h) {
  return h->have_aff && h->aff_h.svc_class != nullptr && (h->ctx.preds & KSIM_P_SERVICE_AFFINITY);
}
// Either of them.
inline bool ksim_rt_launch_tables(const ksim_handle* h) { return ksim_rt_aux_on(h) || ksim_rt_svc_lender_on(h); }
// Pod classes with more than KSIM_MAX_RCLASS reduce classes (the launch form's wide decision).
bool wide_k(const ksim_handle* h, int32_t cls);
int ksim_rt_check_launch_ctx(ksim_handle* h, const KsimCtx& c, int grid, const char* where);
bool ksim_rt_range_wide(const ksim_handle* h, int64_t first, int64_t count);
// err bit 128 (a pod read disagreeing service-affinity labels): clear it, KSIM_E_UNSUPPORTED.
int ksim_rt_svc_refusal(ksim_handle* h);
