// ksim_cache.cpp — the per-pod drop-in entry points and the scheduler-cache event mirror of
// include/ksim.h (ksim_schedule_one, ksim_pod_add / remove, ksim_node_add / update / remove,
// ksim_assume).
//
// Reference surface being served:
//   ScheduleAlgorithm.Schedule           algorithm/scheduler_interface.go:52-65
//   Scheduler.schedule / assume          scheduler.go:188-204, 366-397
//   cache.AssumePod / AddPod / RemovePod schedulercache/cache.go:125, 230, 292
//   cache.AddNode / UpdateNode / Remove  schedulercache/cache.go:354, 366, 378
//   NodeInfo.AddPod / RemovePod / SetNode schedulercache/node_info.go:318-341, 343-390, 429-448
//
// A Schedule call is one scan launch (ksim_scan_kernel, the launch-mode kernel) over the
// resident table against a staged pod descriptor: the pod, its ports / scalars and the result
// block live in one pinned host block mapped into the device's address space, so the kernel reads
// the pod over the bus and writes node, fit count, FitError histogram, error word and
// lastNodeIndex back the same way — one launch and one stream sync per call, no copies.  Node
// events relayout the table in one kernel (rows stay in name-rank order).
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <condition_variable>
#include <mutex>

#include "ksim_handle.h"
#include "ksim_cache.h"

namespace {

// staging layout on the device (and its pinned host mirror)
constexpr size_t STG_CURSOR = 0;
constexpr size_t STG_RES = 16;
constexpr size_t STG_POD = STG_RES + ((KSIM_RES_WORDS * 4 + 15) / 16) * 16;
constexpr size_t STG_PORTS = STG_POD + sizeof(ksim_pod);

// KSIM_CACHE_PROFILE=1 (diagnostic): ksim_schedule_one's host checks + staging, launch calls,
// stream wait, result handling, in ns, printed at exit
struct OneProfile {
  int64_t ns[4] = {0, 0, 0, 0};
  int64_t calls = 0;
  ~OneProfile() {
    if (calls)
      fprintf(stderr, "[ksim schedule_one profile] %lld calls, us/call: checks+staging %.1f launch %.1f wait %.1f result %.1f\n",
              (long long)calls, ns[0] / 1e3 / calls, ns[1] / 1e3 / calls, ns[2] / 1e3 / calls, ns[3] / 1e3 / calls);
  }
};
OneProfile g_one_prof;
bool one_profile() {
  static const bool on = getenv("KSIM_CACHE_PROFILE") && atoi(getenv("KSIM_CACHE_PROFILE")) != 0;
  return on;
}
int64_t g_one_seen = 0;
struct OneClock {
  bool on = one_profile() && g_one_seen++ >= (getenv("KSIM_CACHE_PROFILE_SKIP") ? atoll(getenv("KSIM_CACHE_PROFILE_SKIP")) : 0);
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void lap(int k) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    g_one_prof.ns[k] += std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count();
    t = now;
  }
};

int ensure_staging(ksim_handle* h, int32_t n_ports, int32_t n_scalars) {
  const size_t need = STG_PORTS + (size_t)n_ports * 8 + (size_t)n_scalars * sizeof(ksim_scalar_req) +
                      (size_t)KSIM_PK_WORDS(KSIM_MAX_SCALAR, 0) * 8;
  if (h->stg_host && h->stg_cap >= need) return KSIM_OK;
  const size_t cap = std::max<size_t>(need * 2, 4096);
  char* hst = nullptr;
  HIPCHK(h, hipHostMalloc((void**)&hst, cap, hipHostMallocMapped));
  char* d = nullptr;
  HIPCHK(h, hipHostGetDevicePointer((void**)&d, hst, 0));
  if (h->stg_host) {  // every earlier call has synchronised its stream
    HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
    (void)hipHostFree(h->stg_host);
  }
  memset(hst, 0, cap);
  h->stg_dev = d;
  h->stg_host = hst;
  h->stg_cap = cap;
  h->res_dev = reinterpret_cast<int32_t*>(d + STG_RES);
  h->res_host = reinterpret_cast<int32_t*>(hst + STG_RES);
  return KSIM_OK;
}

// The pod as the per-pod kernels take it: offsets rebased to its own arrays, its reduce-class
// dimensions in reserved[] (as ksim_launch_pod_k does for the queue).
ksim_pod staged_pod(const ksim_handle* h, const ksim_pod& pod) {
  ksim_pod p = pod;
  p.port_off = 0;
  p.scalar_off = 0;
  p.reserved[0] = h->ctx.w[KSIM_W_TAINT_TOLERATION] ? h->h_n_tt[p.cls] : 1;
  p.reserved[1] = h->ctx.use_na ? h->h_n_na[p.cls] : 1;
  return p;
}

// Stage one pod: {cursor = 0, zeroed result block, pod (offsets rebased to the staged arrays),
// ports, scalars} in one copy, and the context that points the scan / commit kernels at it.
int stage_pod(ksim_handle* h, const ksim_pod& pod, const uint64_t* ports, const ksim_scalar_req* scalars,
              KsimCtx* cs) {
  int rc = ensure_staging(h, pod.port_cnt, pod.scalar_cnt);
  if (rc) return rc;
  char* hs = h->stg_host;
  memset(hs, 0, STG_POD);
  const ksim_pod p = staged_pod(h, pod);
  memcpy(hs + STG_POD, &p, sizeof p);
  const size_t pb = (size_t)pod.port_cnt * 8, sb = (size_t)pod.scalar_cnt * sizeof(ksim_scalar_req);
  if (pb) memcpy(hs + STG_PORTS, ports + pod.port_off, pb);
  if (sb) memcpy(hs + STG_PORTS + pb, scalars + pod.scalar_off, sb);
  *cs = h->ctx;
  cs->pods = reinterpret_cast<const ksim_pod*>(h->stg_dev + STG_POD);
  cs->pod_ports = reinterpret_cast<const uint64_t*>(h->stg_dev + STG_PORTS);
  cs->pod_scalars = reinterpret_cast<const ksim_scalar_req*>(h->stg_dev + STG_PORTS + pb);
  cs->cursor = reinterpret_cast<int64_t*>(h->stg_dev + STG_CURSOR);
  // the pod and its arrays in the kernel arguments (the mapped copy above serves pods with more
  // host ports than KSIM_ONE_PORTS)
  cs->one = 0;
  if (pod.port_cnt <= KSIM_ONE_PORTS && pod.scalar_cnt <= KSIM_MAX_SCALAR) {
    cs->one = 1;
    cs->one_pod = p;
    if (pb) memcpy(cs->one_ports, ports + pod.port_off, pb);
    if (sb) memcpy(cs->one_scalars, scalars + pod.scalar_off, sb);
  }
  cs->out_node = h->res_dev + KSIM_RES_NODE;
  cs->out_fit = h->res_dev + KSIM_RES_FIT;
  cs->out_reasons = h->res_dev + KSIM_RES_REASONS;
  cs->first = 0;
  cs->end = 1;
  return KSIM_OK;
}

// The node columns, in one place: (address of the ctx pointer, element bytes, slots).
struct ColRef {
  void** p;
  int32_t esz;
  int32_t slots;
};

std::vector<ColRef> node_cols(ksim_handle* h) {
  KsimCtx& c = h->ctx;
  const int32_t S = c.n_scalar, P = c.port_slots;
  return {{(void**)&c.alloc_cpu, 8, 1},    {(void**)&c.alloc_mem, 8, 1},  {(void**)&c.alloc_gpu, 8, 1},
          {(void**)&c.alloc_eph, 8, 1},    {(void**)&c.allowed_pods, 4, 1}, {(void**)&c.flags, 4, 1},
          {(void**)&c.label_set, 4, 1},    {(void**)&c.taint_set, 4, 1},  {(void**)&c.alloc_scalar, 8, S},
          {(void**)&c.req_cpu, 8, 1},      {(void**)&c.req_mem, 8, 1},    {(void**)&c.req_gpu, 8, 1},
          {(void**)&c.req_eph, 8, 1},      {(void**)&c.nz_cpu, 8, 1},     {(void**)&c.nz_mem, 8, 1},
          {(void**)&c.pod_count, 4, 1},    {(void**)&c.req_scalar, 8, S}, {(void**)&c.ports, 8, P},
          {(void**)&c.port_count, 4, 1}};
}

// Copy the chosen columns into fresh buffers of n_new rows (op: KSIM_RELAY_*) and swap them in.
// new_slots: per column, the slot count after (-1 = unchanged).
int relayout(ksim_handle* h, const std::vector<ColRef>& cols, const std::vector<int32_t>& new_slots, int32_t op,
             int64_t idx, int64_t n_new) {
  KsimRelayout r{};
  r.op = op;
  r.n_old = h->ctx.n;
  r.n_new = n_new;
  r.idx = idx;
  std::vector<void*> fresh(cols.size(), nullptr);
  for (size_t k = 0; k < cols.size(); ++k) {
    const int32_t ds = new_slots[k] < 0 ? cols[k].slots : new_slots[k];
    int rc;
    if (cols[k].esz == 8) {
      uint64_t* q;
      rc = dev_alloc(h, &q, (size_t)ds * n_new);
      fresh[k] = q;
    } else {
      uint32_t* q;
      rc = dev_alloc(h, &q, (size_t)ds * n_new);
      fresh[k] = q;
    }
    if (rc) {
      for (void* q : fresh) dev_free(h, q);
      return rc;
    }
    r.col[r.ncol++] = KsimRelayCol{*cols[k].p, fresh[k], cols[k].esz, cols[k].slots, ds, 0};
  }
  hipError_t e = ksim_launch_relayout(&r, ksim_stream(h));
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "relayout launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  for (size_t k = 0; k < cols.size(); ++k) {
    dev_free(h, *cols[k].p);
    *cols[k].p = fresh[k];
  }
  return KSIM_OK;
}

// Grow the slot-major port column to `slots` slots per node (existing keys keep their slots).
int grow_port_slots(ksim_handle* h, int32_t slots) {
  KsimCtx& c = h->ctx;
  if (slots <= c.port_slots) return KSIM_OK;
  if (slots > 4096) return ksim_fail(h, KSIM_E_OVERFLOW, "a node would hold more than 4096 host ports");
  std::vector<ColRef> cols{{(void**)&c.ports, 8, c.port_slots}};
  int rc = relayout(h, cols, {slots}, KSIM_RELAY_SAME, 0, c.n);
  if (rc) return rc;
  c.port_slots = slots;
  ksim_rt_invalidate_layout(h);
  return KSIM_OK;
}

// The node table can take `need` more distinct host ports on its fullest node: otherwise
// measure the real maximum and, if still short, grow the port column geometrically.
int ensure_port_room(ksim_handle* h, int32_t need) {
  KsimCtx& c = h->ctx;
  if (need <= 0 || h->port_bound + need <= c.port_slots) return KSIM_OK;
  if (c.n > 0) {
    int rc = ensure_staging(h, 0, 0);
    if (rc) return rc;
    hipError_t e = ksim_launch_port_max(c.port_count, c.n, h->res_dev + KSIM_RES_STATUS, ksim_stream(h));
    if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "port max: %s", hipGetErrorString(e));
    HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
    h->port_bound = h->res_host[KSIM_RES_STATUS];
  } else {
    h->port_bound = 0;
  }
  if (h->port_bound + need <= c.port_slots) return KSIM_OK;
  return grow_port_slots(h, (int32_t)std::max<int64_t>({(int64_t)c.port_slots * 2, h->port_bound + need, 4}));
}

int check_ready(ksim_handle* h, const char* where) {
  if (!h) return ksim_fail(h, KSIM_E_INVAL, "%s: null handle", where);
  if (!h->have_nodes || !h->have_classes) return ksim_fail(h, KSIM_E_STATE, "%s: load nodes and classes first", where);
  if (h->shard.world > 1) return ksim_fail(h, KSIM_E_UNSUPPORTED, "%s: not available on a node-sharded handle", where);
  HIPCHK(h, hipSetDevice(h->device));
  return KSIM_OK;
}

// A node event: the affinity tables' per-node domains no longer describe the table.
void node_event(ksim_handle* h) {
  if (h->have_aff) h->aff_stale = true;
  if (h->have_vol) h->vol_stale = true;
}

int check_pod_args(ksim_handle* h, const ksim_pod* pod, int32_t n_ports, int32_t n_scalars, const uint64_t* ports,
                   const ksim_scalar_req* scalars, const char* where) {
  if (!pod) return ksim_fail(h, KSIM_E_INVAL, "%s: null pod", where);
  if (n_ports < 0 || n_scalars < 0 || (n_ports && !ports) || (n_scalars && !scalars))
    return ksim_fail(h, KSIM_E_INVAL, "%s: bad port / scalar arrays", where);
  if (pod->port_cnt < 0 || pod->port_off < 0 || (int64_t)pod->port_off + pod->port_cnt > n_ports)
    return ksim_fail(h, KSIM_E_INVAL, "%s: port range out of bounds", where);
  return KSIM_OK;
}

bool ksim_is_aff_host(const ksim_handle* h, const ksim_pod& p) {
  return h->have_aff && (p.aff_ident || p.aff_class);
}

int after_commit(ksim_handle* h, int32_t port_cnt, const int32_t* r = nullptr) {
  if (!r) r = h->res_host;
  h->tree_valid = false;  // the trees are maintained by the tree kernel only
  const int32_t status = r[KSIM_RES_STATUS];
  if (status & 2)  // the committing kernel reported the row's port count: the bound stays exact
    h->port_bound = std::max<int64_t>(h->port_bound, (int64_t)(status >> 8));
  else
    h->port_bound += port_cnt;
  if (status & 1) h->pfast_off = true;  // keep the fast kernels' float64 range
  const int32_t err = r[KSIM_RES_ERR];  // written by the committing kernel
  if (err & 1) return ksim_fail(h, KSIM_E_OVERFLOW, "a node's host-port or volume slots overflowed (raise port_slots / vol_slots)");
  if (err & ~1) return ksim_fail(h, KSIM_E_DEVICE, "device consistency error 0x%x", err);
  return KSIM_OK;
}

// ---- the resident per-pod service (ksim_serve_kernel in ksim_kernels.hip) ----
// A block votes to leave after SERVE_IDLE_TICKS without a message; the grid leaves when the vote
// is unanimous (KSIM_SERVE_ST_*, ksim_common.h), and a message the grid left before taking is
// served by a fresh launch that finds it in the mailbox.  KSIM_SERVE=0: per-pod launches only.
// KSIM_SERVE_IDLE_MS overrides the idle bound (tests).
constexpr int64_t SERVE_WAIT_NS = 10000000000ll;  // an answer's bound (the kernel's spins end in 2 s)
constexpr int SERVE_RELAUNCHES = 4;               // relaunches for one message (each finds it waiting)

int64_t now_ns() {
  return std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

uint64_t serve_idle_ticks() {
  static const uint64_t t = getenv("KSIM_SERVE_IDLE_MS") ? strtoull(getenv("KSIM_SERVE_IDLE_MS"), nullptr, 10) * 100000ull
                                                         : 20000000ull;  // 200 ms of s_memrealtime (100 MHz)
  return t;
}

bool serve_wanted(const ksim_handle* h) {
  static const bool env_off = getenv("KSIM_SERVE") && getenv("KSIM_SERVE")[0] == '0';
  return !env_off && !h->serve_off;
}

size_t serve_stage_bytes(int grid) {
  return (size_t)grid * (sizeof(ksim_pod) + 8 * KSIM_ONE_PORTS + sizeof(ksim_scalar_req) * KSIM_MAX_SCALAR);
}

// ---- the device gate (KsimGate, ksim_handle.h) and the handles whose resident kernel runs ----
// Two classes of sections that exclude each other but not themselves: the resident kernels' calls
// (shared) and the co-resident launches (exclusive towards the former only: node-sharded ranks on
// one device run their kernels side by side, and waiting for each other is their protocol).  A
// waiting co-resident launch holds back new resident sections, so a stream of per-pod calls cannot
// starve it.
struct DeviceGate {
  std::mutex mu;
  std::condition_variable cv;
  int n_serve = 0, n_batch = 0, n_batch_waiting = 0;
  std::mutex stop_mu;  // one stopper of other handles' resident kernels at a time
  std::mutex reg_mu;
  std::vector<ksim_handle*> live;
};
DeviceGate& device_gate(int dev) {
  static DeviceGate g[64];
  return g[dev & 63];
}
thread_local int8_t t_gate_hold[64];  // per device: 0, 1 shared, 2 exclusive (this thread)

void serve_register(ksim_handle* h, bool on) {
  DeviceGate& g = device_gate(h->device);
  std::lock_guard<std::mutex> lk(g.reg_mu);
  g.live.erase(std::remove(g.live.begin(), g.live.end(), h), g.live.end());
  if (on) g.live.push_back(h);
}

// The launch named in KsimServeBox::left: the grid left by its idle vote.
bool serve_left(const ksim_handle* h) {
  const uint64_t l = __atomic_load_n(&h->serve_box->left, __ATOMIC_ACQUIRE);
  return (uint32_t)(l >> 32) == h->serve_launch_id;
}

// The grid left by its idle vote: drain the stream (its last blocks are on their way out).
// After the resident kernel drained: an undo it was told of but did not apply (the grid left
// before its record's block took the message) is done by a launch.
int tent_drained(ksim_handle* h) {
  if (!h->tent.undo_inflight) return KSIM_OK;
  h->tent.undo_inflight = false;
  if ((uint32_t)__atomic_load_n(&h->serve_box->undo_ack, __ATOMIC_ACQUIRE) == h->tent.rec.seq) return KSIM_OK;
  hipError_t e = ksim_launch_undo(&h->ctx, &h->tent.rec, h->stream_raw);
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "undo launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipStreamSynchronize(h->stream_raw));
  h->tent_stats[2] += 1;
  return KSIM_OK;
}

int serve_reap(ksim_handle* h) {
  h->serve_live.store(false, std::memory_order_release);
  serve_register(h, false);
  HIPCHK(h, hipStreamSynchronize(h->stream_raw));
  h->serve_stats[3] += 1;
  return tent_drained(h);
}

// Launch the resident kernel over the current context; seq0 = the newest message already
// handled (a relaunch for an untaken message passes the one before it).
int serve_launch(ksim_handle* h, int npt, int grid, uint64_t seq0) {
  if (!h->serve_box) {
    KsimServeBox* b = nullptr;
    HIPCHK(h, hipHostMalloc((void**)&b, sizeof(KsimServeBox), hipHostMallocMapped | hipHostMallocCoherent));
    memset((void*)b, 0, sizeof *b);
    KsimServeBox* d = nullptr;
    HIPCHK(h, hipHostGetDevicePointer((void**)&d, b, 0));
    h->serve_box = b;
    h->serve_box_dev = d;
  }
  if (!h->serve_state) {
    int rc = dev_alloc(h, &h->serve_state, 1);
    if (rc) return rc;
  }
  if (h->serve_grid < grid || !h->serve_stage) {
    dev_free(h, h->serve_stage);
    h->serve_stage = nullptr;
    int rc = dev_alloc(h, &h->serve_stage, serve_stage_bytes(grid));
    if (rc) return rc;
  }
  KsimCtx cs = h->ctx;
  cs.one = 0;  // the pod comes from the mailbox, through each block's staging slot
  cs.pods = reinterpret_cast<const ksim_pod*>(h->serve_stage);
  cs.pod_ports = reinterpret_cast<const uint64_t*>(h->serve_stage + (size_t)grid * sizeof(ksim_pod));
  cs.pod_scalars = reinterpret_cast<const ksim_scalar_req*>(h->serve_stage + (size_t)grid * (sizeof(ksim_pod) + 8 * KSIM_ONE_PORTS));
  cs.chunk = (int64_t)KSIM_BLOCK * npt;
  cs.collect = 1;
  cs.first = 0;
  cs.end = 1;
  cs.pick = h->pick_words;
  // (unused: the resident form answers in KsimServeBox::ans; the staging result block keeps the
  // context's pointers valid for the pre-launch check)
  int rc0 = ensure_staging(h, 0, 0);
  if (rc0) return rc0;
  cs.out_node = h->res_dev + KSIM_RES_NODE;
  cs.out_fit = h->res_dev + KSIM_RES_FIT;
  cs.out_reasons = h->res_dev + KSIM_RES_REASONS;
  int rc = ksim_rt_check_launch_ctx(h, cs, grid, "ksim_schedule_one (resident)");
  if (rc) return rc;
  HIPCHK(h, hipMemsetAsync(h->serve_state, 0, 8, h->stream_raw));
  KsimServeArgs a{};
  a.box = h->serve_box_dev;
  a.state = h->serve_state;
  a.seq0 = seq0;
  a.idle_ticks = serve_idle_ticks();
  a.ctr0 = h->ctr_host;
  a.ctr0_valid = h->ctr_known ? 1u : 0u;
  if (++h->serve_launch_id == 0) h->serve_launch_id = 1;  // (0 = the `left` word's initial value)
  a.launch_id = h->serve_launch_id;
  h->serve_aux = ksim_rt_aux_on(h);
  hipError_t e = ksim_launch_serve(&cs, &a, npt, grid, h->serve_aux ? 1 : 0, h->stream_raw);
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "resident per-pod kernel launch: %s", hipGetErrorString(e));
  h->serve_live.store(true, std::memory_order_release);
  serve_register(h, true);
  h->serve_shared = false;  // (the launch itself acquires)
  h->serve_base = h->ctx;
  h->serve_npt = npt;
  h->serve_grid = grid;
  h->serve_stats[0] += 1;
  return KSIM_OK;
}

// Write one message into the mailbox (every word tagged with its number: KSIM_SERVE_MSG_WORDS).
uint64_t serve_write(ksim_handle* h, int32_t type, const ksim_pod* p, const uint64_t* ports,
                     const ksim_scalar_req* scalars, int32_t no_commit, int64_t node, uint32_t tag, int32_t sync) {
  uint32_t w[KSIM_SERVE_MSG_WORDS] = {};
  w[KSIM_SERVE_W_TYPE] = (uint32_t)type;
  w[KSIM_SERVE_W_NOCOMMIT] = (uint32_t)no_commit;
  w[KSIM_SERVE_W_TAG] = tag;
  w[KSIM_SERVE_W_SYNC] = (uint32_t)sync;
  w[KSIM_SERVE_W_NODE] = (uint32_t)(uint64_t)node;
  w[KSIM_SERVE_W_NODE + 1] = (uint32_t)((uint64_t)node >> 32);
  w[KSIM_SERVE_W_TENT_SEQ] = h->tent.rec.seq;
  w[KSIM_SERVE_W_TENT_ACT] = (uint32_t)h->tent.act;
  if (p) {
    memcpy(w + KSIM_SERVE_W_POD, p, sizeof *p);
    if (p->port_cnt) memcpy(w + KSIM_SERVE_W_PORTS, ports, (size_t)p->port_cnt * 8);
    if (p->scalar_cnt) memcpy(w + KSIM_SERVE_W_SCALARS, scalars, (size_t)p->scalar_cnt * sizeof(ksim_scalar_req));
  }
  const uint64_t seq = ++h->serve_seq;
  const uint64_t tg = (uint64_t)(uint32_t)seq << 32;
  uint64_t* m = h->serve_box->msg;
  for (int k = 0; k < KSIM_SERVE_MSG_WORDS; ++k) __atomic_store_n(&m[k], tg | w[k], __ATOMIC_RELAXED);
  return seq;
}

// The answer to message seq, when every word the host reads carries its number (node, fit,
// status, error, lastNodeIndex; the reasons of a FitError).
bool serve_answer(const ksim_handle* h, uint64_t seq, int32_t* r, bool tent = false) {
  const uint32_t s = (uint32_t)seq;
  const uint64_t* a = h->serve_box->ans;
  auto word = [&](int k) {
    const uint64_t w = __atomic_load_n(&a[k], __ATOMIC_ACQUIRE);
    r[k] = (int32_t)(uint32_t)w;
    return (uint32_t)(w >> 32) == s;
  };
  for (int k : {KSIM_RES_NODE, KSIM_RES_FIT, KSIM_RES_STATUS, KSIM_RES_ERR, KSIM_RES_CTR, KSIM_RES_CTR + 1})
    if (!word(k)) return false;
  if (r[KSIM_RES_NODE] == -1) {
    for (int k = 0; k < KSIM_NREASONS; ++k)
      if (!word(KSIM_RES_REASONS + k)) return false;
  } else {
    memset(r + KSIM_RES_REASONS, 0, KSIM_NREASONS * 4);
    if (tent && r[KSIM_RES_NODE] >= 0)  // the row's port count and flags before the commit
      for (int k = 0; k < 2; ++k)
        if (!word(KSIM_RES_REASONS + k)) return false;
  }
  return true;
}

// The resident kernel cannot serve this handle any more: per-pod launches from now on.
int serve_fail(ksim_handle* h, const char* fmt, ...) {
  char msg[256];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(msg, sizeof msg, fmt, ap);
  va_end(ap);
  h->serve_off = true;
  if (h->serve_live.load() && !serve_left(h)) (void)ksim_serve_stop(h);
  else if (h->serve_live.load()) (void)serve_reap(h);
  return ksim_fail(h, KSIM_E_DEVICE, "%s", msg);
}

// Post one message and wait for its answer (r: KSIM_RES_WORDS result words).  Called under the
// device gate (shared).
int serve_post(ksim_handle* h, int32_t type, const ksim_pod& p, const uint64_t* ports, const ksim_scalar_req* scalars,
               int32_t no_commit, int64_t node, uint32_t tag, int32_t* r) {
  const bool tent = type == KSIM_SERVE_SCHEDULE && no_commit == KSIM_SERVE_TENTATIVE;
  // the system-scope acquire only after commits of state other blocks read (inter-pod affinity /
  // service counts, volumes); KSIM_SERVE_LIGHT=0: before every message
  static const bool light_off = getenv("KSIM_SERVE_LIGHT") && getenv("KSIM_SERVE_LIGHT")[0] == '0';
  // serve_shared: a commit of such state since the last SCHEDULE message.  Every block takes every
  // SCHEDULE message (each publishes records for it), but a block may skip an ASSUME onto another
  // block's node, so the pending acquire is cleared only by a SCHEDULE message.
  const bool shared = ksim_is_aff_host(h, p) || p.vol_class != 0;
  const int32_t sync = h->serve_shared || light_off ? KSIM_SERVE_SYNC_ACQUIRE : 0;
  h->serve_shared = type == KSIM_SERVE_SCHEDULE ? shared : (h->serve_shared || shared);
  const uint64_t seq = serve_write(h, type, &p, ports, scalars, no_commit, node, tag, sync);
  h->serve_stats[1] += 1;
  int64_t t0 = now_ns(), next_check = t0 + 1000000;  // every 1 ms: is the kernel still there?
  int relaunches = 0;
  for (uint64_t spins = 0; !serve_answer(h, seq, r, tent); ++spins) {
    __builtin_ia32_pause();
    if ((spins & 63) != 63) continue;
    if (serve_left(h)) {
      // the grid agreed to leave before any block took this message (a block that voted takes a
      // message only after withdrawing its vote, which fails once the vote is unanimous), so the
      // message is still whole in the mailbox: a fresh launch takes it as its first
      if (serve_answer(h, seq, r, tent)) break;
      if (++relaunches > SERVE_RELAUNCHES)
        return serve_fail(h, "resident per-pod kernel: message %llu not taken after %d relaunches", (unsigned long long)seq,
                          SERVE_RELAUNCHES);
      int rc = serve_reap(h);
      if (rc) return rc;
      h->serve_stats[4] += 1;
      if ((rc = serve_launch(h, h->serve_npt, h->serve_grid, seq - 1))) return rc;
      t0 = now_ns();
      next_check = t0 + 1000000;
      continue;
    }
    const int64_t t = now_ns();
    if (t < next_check) continue;
    next_check = t + 1000000;
    const bool gone = hipStreamQuery(h->stream_raw) == hipSuccess;
    if (serve_answer(h, seq, r, tent) || serve_left(h)) continue;  // (the loop's checks take it from here)
    if (gone || t - t0 > SERVE_WAIT_NS)
      return serve_fail(h, "resident per-pod kernel %s (message %llu)", gone ? "left before answering" : "did not answer",
                        (unsigned long long)seq);
  }
  // lastNodeIndex: selectHost bumps it exactly when two or more nodes fit; an ASSUME leaves it
  const int32_t err = r[KSIM_RES_ERR];
  const uint64_t ctr = (uint64_t)(uint32_t)r[KSIM_RES_CTR] | ((uint64_t)(uint32_t)r[KSIM_RES_CTR + 1] << 32);
  if (r[KSIM_RES_NODE] != INT32_MIN && err == 0) {
    if (h->ctr_known) {
      const uint64_t want = h->ctr_host + (type == KSIM_SERVE_SCHEDULE && r[KSIM_RES_FIT] >= 2 ? 1 : 0);
      if (ctr != want)
        return serve_fail(h, "resident per-pod kernel answered lastNodeIndex %llu, expected %llu (message %llu)",
                          (unsigned long long)ctr, (unsigned long long)want, (unsigned long long)seq);
    }
    h->ctr_host = ctr;
    h->ctr_known = true;
  }
  // the decision on the last tentative commit went out with this message: acknowledged yet?
  if (h->tent.undo_inflight && (uint32_t)__atomic_load_n(&h->serve_box->undo_ack, __ATOMIC_ACQUIRE) == h->tent.rec.seq)
    h->tent.undo_inflight = false;
  if (tent && r[KSIM_RES_NODE] >= 0 && err == 0) {  // a tentative commit: the record's host copy
    h->tent.live = true;
    h->tent.launch = h->serve_launch_id;  // (the launch that answered: a relaunch's, when it served it)
    h->tent.act = KSIM_TENT_NONE;
    h->tent.rec.node = r[KSIM_RES_NODE];
    h->tent.rec.seq = (uint32_t)seq;
    h->tent.rec.cnt0 = r[KSIM_RES_REASONS];
    h->tent.rec.fl0 = (uint32_t)r[KSIM_RES_REASONS + 1];
    h->tent.rec.P = p;
    h->tent.rec.valid = 1;
    for (int32_t k = 0; k < p.scalar_cnt; ++k) h->tent.rec.sc[k] = scalars[k];
    for (int32_t k = 0; k < p.port_cnt; ++k) h->tent.ports[k] = ports[k];
    memcpy(h->tent.res, r, sizeof h->tent.res);
    h->tent_stats[0] += 1;
  }
  return KSIM_OK;
}

// The resident kernel serves the current context with this geometry: (re)start it when not.
// Called under the device gate (shared).
int serve_ready(ksim_handle* h, int npt, int grid) {
  if (h->serve_live.load()) {
    if (serve_left(h)) {  // the grid left by its idle vote while the host was away
      int rc = serve_reap(h);
      if (rc) return rc;
    } else if (h->serve_npt != npt || h->serve_grid != grid || h->serve_aux != ksim_rt_aux_on(h) ||
               memcmp(&h->ctx, &h->serve_base, sizeof(KsimCtx)) != 0) {
      int rc = ksim_serve_stop(h);
      if (rc) return rc;
    }
  }
  if (!h->serve_live.load()) return serve_launch(h, npt, grid, h->serve_seq);
  return KSIM_OK;
}

void pack_row(const KsimCtx& c, const ksim_node_row* r, std::vector<uint64_t>& pk) {
  pk.assign(KSIM_PK_WORDS(c.n_scalar, c.port_slots), 0);
  pk[KSIM_PK_ALLOC + 0] = (uint64_t)r->alloc_cpu;
  pk[KSIM_PK_ALLOC + 1] = (uint64_t)r->alloc_mem;
  pk[KSIM_PK_ALLOC + 2] = (uint64_t)r->alloc_gpu;
  pk[KSIM_PK_ALLOC + 3] = (uint64_t)r->alloc_eph;
  pk[KSIM_PK_ALLOWED] = (uint64_t)(uint32_t)r->allowed_pods;
  pk[KSIM_PK_FLAGS] = r->flags;
  pk[KSIM_PK_LABEL] = (uint64_t)(uint32_t)r->label_set;
  pk[KSIM_PK_TAINT] = (uint64_t)(uint32_t)r->taint_set;
  pk[KSIM_PK_REQ + 0] = (uint64_t)r->req_cpu;
  pk[KSIM_PK_REQ + 1] = (uint64_t)r->req_mem;
  pk[KSIM_PK_REQ + 2] = (uint64_t)r->req_gpu;
  pk[KSIM_PK_REQ + 3] = (uint64_t)r->req_eph;
  pk[KSIM_PK_NZ + 0] = (uint64_t)r->nz_cpu;
  pk[KSIM_PK_NZ + 1] = (uint64_t)r->nz_mem;
  pk[KSIM_PK_COUNT] = (uint64_t)(uint32_t)r->pod_count;
  pk[KSIM_PK_PORTCNT] = (uint64_t)(uint32_t)r->port_count;
  for (int32_t k = 0; k < c.n_scalar; ++k) {
    pk[KSIM_PK_SCALAR + k] = r->alloc_scalar ? (uint64_t)r->alloc_scalar[k] : 0;
    pk[KSIM_PK_SCALAR + c.n_scalar + k] = r->req_scalar ? (uint64_t)r->req_scalar[k] : 0;
  }
  for (int32_t k = 0; k < r->port_count; ++k) pk[KSIM_PK_SCALAR + 2 * c.n_scalar + k] = r->ports[k];
}

int check_row(ksim_handle* h, const ksim_node_row* r, bool full, const char* where) {
  if (!r) return ksim_fail(h, KSIM_E_INVAL, "%s: null row", where);
  if (r->label_set < 0 || r->label_set >= h->n_label_sets || r->taint_set < 0 || r->taint_set >= h->n_taint_sets)
    return ksim_fail(h, KSIM_E_INVAL, "%s: label / taint set id outside the loaded class tables (reload them first)", where);
  if (full && (r->port_count < 0 || (r->port_count && !r->ports) || r->pod_count < 0))
    return ksim_fail(h, KSIM_E_INVAL, "%s: bad pod / port count", where);
  return KSIM_OK;
}

// A node row inside the fast kernels' exact float64 range (ksim_pfast.hip, ksim_tree.hip)?
bool row_exact(const ksim_node_row* r, bool full) {
  const int64_t lim = (int64_t)1 << 48;
  for (int64_t v : {r->alloc_cpu, r->alloc_mem})
    if (v < 0 || v >= lim) return false;
  if (full)
    for (int64_t v : {r->req_cpu, r->req_mem, r->nz_cpu, r->nz_mem})
      if (v < 0 || v >= lim) return false;
  return true;
}

int set_row(ksim_handle* h, int64_t index, const ksim_node_row* row, bool full) {
  std::vector<uint64_t> pk;
  pack_row(h->ctx, row, pk);
  int rc = ensure_staging(h, (int32_t)pk.size(), 0);
  if (rc) return rc;
  memcpy(h->stg_host + STG_PORTS, pk.data(), pk.size() * 8);  // read by the kernel through the mapping
  hipError_t e = ksim_launch_set_row(&h->ctx, index, reinterpret_cast<const uint64_t*>(h->stg_dev + STG_PORTS), full ? 1 : 0,
                                     ksim_stream(h));
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "set_row launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  if (!row_exact(row, full)) h->pfast_off = true;
  return KSIM_OK;
}

int node_shift(ksim_handle* h, int32_t op, int64_t index) {
  KsimCtx& c = h->ctx;
  const std::vector<ColRef> cols = node_cols(h);
  const int64_t n_new = op == KSIM_RELAY_INSERT ? c.n + 1 : c.n - 1;
  int rc = relayout(h, cols, std::vector<int32_t>(cols.size(), -1), op, index, n_new);
  if (rc) return rc;
  c.n = n_new;
  if (h->have_pods && h->n_pods) {
    hipError_t e = ksim_launch_remap_hosts(h->d_pods, h->n_pods, index, op, ksim_stream(h));
    if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "remap launch: %s", hipGetErrorString(e));
    HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  }
  ksim_rt_invalidate_layout(h);
  return KSIM_OK;
}

}  // namespace

KsimGate::KsimGate(ksim_handle* h, bool exclusive) {
  if (!h) return;
  dev = h->device & 63;
  if (t_gate_hold[dev]) return;  // held by this thread already (a co-resident launch's own resident stop)
  DeviceGate& g = device_gate(dev);
  {
    std::unique_lock<std::mutex> lk(g.mu);
    if (!exclusive) {
      g.cv.wait(lk, [&] { return g.n_batch == 0 && g.n_batch_waiting == 0; });
      g.n_serve += 1;
      mode = 1;
      t_gate_hold[dev] = 1;
      return;
    }
    g.n_batch_waiting += 1;
    g.cv.wait(lk, [&] { return g.n_serve == 0; });
    g.n_batch_waiting -= 1;
    g.n_batch += 1;
  }
  mode = 2;
  t_gate_hold[dev] = 2;
  // no handle's call is inside its resident section now: stop the other handles' kernels here
  std::lock_guard<std::mutex> sl(g.stop_mu);
  std::vector<ksim_handle*> others;
  {
    std::lock_guard<std::mutex> lk(g.reg_mu);
    for (ksim_handle* x : g.live)
      if (x != h) others.push_back(x);
  }
  for (ksim_handle* x : others) (void)ksim_serve_stop(x);
}

KsimGate::~KsimGate() {
  if (!mode) return;
  DeviceGate& g = device_gate(dev);
  t_gate_hold[dev] = 0;
  std::lock_guard<std::mutex> lk(g.mu);
  if (mode == 2) g.n_batch -= 1;
  else g.n_serve -= 1;
  g.cv.notify_all();
}

void ksim_serve_forget(ksim_handle* h) { serve_register(h, false); }

int ksim_tent_undo(ksim_handle* h) {
  if (!h->tent.live) return KSIM_OK;
  h->tent.live = false;
  h->tent_stats[1] += 1;
  const ksim_pod& P = h->tent.rec.P;
  const bool shared = ksim_is_aff_host(h, P) || P.vol_class != 0;
  if (h->serve_live.load() && h->tent.launch == h->serve_launch_id && !serve_left(h)) {
    if (!shared) {
      // the kernel that holds the record runs: the next message (a stop's EXIT included) carries
      // the undo, applied by the record's block before anything reads the row
      h->tent.act = KSIM_TENT_UNDO;
      h->tent.undo_inflight = true;
      return KSIM_OK;
    }
    // mounts / affinity counts other blocks read: an UNDO message of its own, answered once the
    // undo is released (the next message acquires)
    KsimGate gate(h, false);
    h->tent.act = KSIM_TENT_UNDO;
    int32_t r[KSIM_RES_WORDS];
    int rc = serve_post(h, KSIM_SERVE_UNDO, P, h->tent.ports, h->tent.rec.sc, 0, h->tent.rec.node, 0, r);
    h->tent.act = KSIM_TENT_NONE;
    if (rc) return rc;
    if (r[KSIM_RES_ERR]) return ksim_fail(h, KSIM_E_DEVICE, "device consistency error 0x%x (undo)", r[KSIM_RES_ERR]);
    if (r[KSIM_RES_STATUS] == 1) return KSIM_OK;
    // no block held the record (a relaunch served the message): the launch below
  }
  // the record left with an earlier launch: undo by a launch on the quiet stream
  h->tent.act = KSIM_TENT_NONE;
  if (h->serve_live.load()) {
    int rc = serve_left(h) ? serve_reap(h) : ksim_serve_stop(h);
    if (rc) return rc;
  }
  hipError_t e = ksim_launch_undo(&h->ctx, &h->tent.rec, h->stream_raw);
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "undo launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipStreamSynchronize(h->stream_raw));
  h->tent_stats[2] += 1;
  return KSIM_OK;
}

// ksim_pod_add right after a tentative commit, naming the same pod and node: the commit stands.
static bool tent_confirms(ksim_handle* h, int64_t node, const ksim_pod& pod, const uint64_t* ports, const ksim_scalar_req* scalars) {
  if (!h->tent.live || node != h->tent.rec.node || pod.port_cnt > KSIM_ONE_PORTS || pod.scalar_cnt > KSIM_MAX_SCALAR) return false;
  ksim_pod a = staged_pod(h, pod), b = h->tent.rec.P;
  a.host = b.host = -1;  // (spec.nodeName plays no part in the commit)
  if (memcmp(&a, &b, sizeof a) != 0) return false;
  for (int32_t k = 0; k < pod.port_cnt; ++k)
    if (ports[pod.port_off + k] != h->tent.ports[k]) return false;
  for (int32_t k = 0; k < pod.scalar_cnt; ++k)
    if (memcmp(&scalars[pod.scalar_off + k], &h->tent.rec.sc[k], sizeof(ksim_scalar_req)) != 0) return false;
  return true;
}

int ksim_serve_stop(ksim_handle* h) {
  if (!h->serve_live.load(std::memory_order_acquire)) return KSIM_OK;
  KsimGate gate(h, false);
  if (!h->serve_live.load()) return KSIM_OK;
  h->serve_live.store(false, std::memory_order_release);  // (first: the drain below goes through the raw stream)
  serve_register(h, false);
  h->serve_stats[2] += 1;
  (void)serve_write(h, KSIM_SERVE_EXIT, nullptr, nullptr, nullptr, 0, -1, 0, 0);
  HIPCHK(h, hipStreamSynchronize(h->stream_raw));
  if (int rc = tent_drained(h)) return rc;
#ifdef KSIM_STAMPS
  uint64_t d[32];
  HIPCHK(h, hipMemcpy(d, h->ctx.dbg + 64, sizeof d, hipMemcpyDeviceToHost));
  HIPCHK(h, hipMemset(h->ctx.dbg + 64, 0, sizeof d));
  static const char* names[11] = {"idle+poll", "copy", "eval", "passA", "publish", "records-wait", "class-stats",
                                  "decision", "owner-select", "commit", "answer"};
  if (d[16 + 1]) {
    fprintf(stderr, "[ksim stamps] serve: %llu block-messages, us per phase (count):", (unsigned long long)d[17]);
    for (int k = 0; k < 11; ++k)
      fprintf(stderr, " %s %.2f (%llu)", names[k], d[k] / 100.0 / std::max<uint64_t>(d[16 + k], 1), (unsigned long long)d[16 + k]);
    fprintf(stderr, " | polls per message %.2f\n", (double)d[11] / std::max<uint64_t>(d[27], 1));
  }
#endif
  return KSIM_OK;
}

void ksim_rt_invalidate_layout(ksim_handle* h) {
  if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
  if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
  for (void* q : {(void*)h->t_leaves, (void*)h->t_levels, (void*)h->t_fit, (void*)h->t_y, (void*)h->sw_dac,
                  (void*)h->sw_dam, (void*)h->sw_yc, (void*)h->sw_ym, (void*)h->mirror})
    dev_free(h, q);
  h->t_leaves = nullptr; h->t_levels = nullptr; h->t_fit = nullptr; h->t_y = nullptr;
  h->sw_dac = h->sw_dam = h->sw_yc = h->sw_ym = nullptr;
  h->mirror = nullptr;
  h->mirror_n = 0;
  h->tree_planned = h->tree_ok = h->tree_valid = false;
}

extern "C" {

int ksim_schedule_one(ksim_handle* h, const ksim_pod* pod, const uint64_t* ports, int32_t n_ports,
                      const ksim_scalar_req* scalars, int32_t n_scalars, int32_t assume, ksim_result* out) {
  OneClock oc;
  if (oc.on) g_one_prof.calls += 1;
  int rc = check_ready(h, "ksim_schedule_one");
  if (rc) return rc;
  if (!out) return ksim_fail(h, KSIM_E_INVAL, "ksim_schedule_one: null result");
  if ((rc = check_pod_args(h, pod, n_ports, n_scalars, ports, scalars, "ksim_schedule_one"))) return rc;
  KsimCtx& c = h->ctx;
  if (c.n == 0) return ksim_fail(h, KSIM_E_NO_NODES, "no nodes available to schedule pods");
  if ((rc = ksim_rt_check_aff(h, "ksim_schedule_one"))) return rc;
  // room for the pod's ports if it is assumed (and at least one slot column to test against)
  if ((assume || c.port_slots == 0) && (rc = ensure_port_room(h, pod->port_cnt))) return rc;
  if ((rc = ksim_rt_check_pod(h, *pod, n_ports, n_scalars, scalars, "ksim_schedule_one"))) return rc;
  // every scratch buffer the launch forms read is allocated (or re-allocated) BEFORE the per-pod
  // context is copied from the handle's, so the copy never holds a freed or null pointer (round 4:
  // an illegal access when the wide decision's wmx / wcnt were re-allocated after the copy)
  const int npt = ksim_rt_pick_npt(c.n);
  const int grid = (int)((c.n + (int64_t)KSIM_BLOCK * npt - 1) / ((int64_t)KSIM_BLOCK * npt));
  if ((rc = ksim_rt_ensure_partials(h, grid))) return rc;
  KsimCtx cs;
  if ((rc = stage_pod(h, *pod, ports, scalars, &cs))) return rc;
  cs.collect = 1;  // the FitError histogram is part of the answer
  cs.no_commit = assume ? 0 : 1;
  // a small cluster: the single-workgroup kernel (every reduction in LDS, no cross-block round
  // trips); measured slower than the multi-block scan at 5,000 nodes (its evaluation has one CU's
  // load bandwidth), so by default only up to 1,024 nodes.  KSIM_ONE_WG=0: never, =1: whenever it fits.
  const int one_npt = ksim_one_npt(c.n);
  const char* ko = getenv("KSIM_ONE_WG");
  const bool one_wg = ko ? ko[0] != '0' : c.n <= 1024;
  if (cs.one && one_npt > 0 && one_wg && (!h->have_aff || h->aff_h.n_zone <= 512) &&
      (!ksim_rt_aux_on(h) || h->aff_h.n_adom <= 512) &&
      cs.one_pod.reserved[0] * cs.one_pod.reserved[1] <= KSIM_MAX_RCLASS) {
    h->res_host[KSIM_RES_NODE] = INT32_MIN;
    if ((rc = ksim_rt_check_launch_ctx(h, cs, 1, "ksim_schedule_one"))) return rc;
    oc.lap(0);
    hipError_t e1 = ksim_launch_one(&cs, one_npt, ksim_stream(h));
    if (e1 != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "one-workgroup launch: %s", hipGetErrorString(e1));
    oc.lap(1);
    HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
    oc.lap(2);
    const int32_t* r = h->res_host;
    memset(out, 0, sizeof *out);
    out->node = r[KSIM_RES_NODE];
    out->fit_nodes = r[KSIM_RES_FIT];
    memcpy(&out->last_node_index, r + KSIM_RES_CTR, 8);
    if (out->node < 0) memcpy(out->reasons, r + KSIM_RES_REASONS, sizeof out->reasons);
    if (assume && out->node >= 0) {
      rc = after_commit(h, pod->port_cnt);
      oc.lap(3);
      return rc;
    }
    if (r[KSIM_RES_ERR] & 128) return ksim_rt_svc_refusal(h);
    if (r[KSIM_RES_ERR]) return ksim_fail(h, KSIM_E_DEVICE, "device consistency error 0x%x", r[KSIM_RES_ERR]);
    return KSIM_OK;
  }
  cs.chunk = (int64_t)KSIM_BLOCK * npt;
  // the pick kernel (<= 64 blocks, co-resident): one tagged-record exchange per reduction and a
  // redundant decision in every block instead of the scan's last-block round trips.  Not for node
  // sharding, more pass-A words than one record holds (4 + spread zones + with the auxiliary
  // priority 3 + its domains <= 64) or scores beyond its 56-bit record words.  KSIM_NO_PICK=1
  // disables it.  (The service-affinity lender check reads only the global counts, which every
  // block sees after the previous commit, as the inter-pod affinity terms do.)
  const char* npk = getenv("KSIM_NO_PICK");
  if (cs.one && grid <= KSIM_PICK_MAXG && !(npk && npk[0] == '1') && c.sh_world <= 1 &&
      cs.one_pod.reserved[0] * cs.one_pod.reserved[1] <= KSIM_MAX_RCLASS &&
      (!h->have_aff || h->aff_h.n_zone + (ksim_rt_aux_on(h) ? 3 + h->aff_h.n_adom : 0) <= KSIM_PICK_ZMAX)) {
    int64_t sw = 0;
    for (int k = 0; k < KSIM_NW; ++k) sw += (c.w[k] > ((int64_t)1 << 40) ? ((int64_t)1 << 50) : c.w[k] * 10);
    if (ksim_rt_aux_on(h)) sw += h->aff_h.aux_w > ((int64_t)1 << 40) ? ((int64_t)1 << 50) : h->aff_h.aux_w * 10;
    if (h->pick_grid != grid || h->pick_npt != npt) {
      h->pick_ok = ksim_pick_coresident(npt, grid) != 0;
      h->serve_fits = ksim_serve_coresident(npt, grid) != 0;
      h->pick_grid = grid;
      h->pick_npt = npt;
      h->pick_clear = true;
    }
    if (sw < ((int64_t)1 << 54) && h->pick_ok) {
      if (!h->pick_words) {
        if ((rc = dev_alloc(h, &h->pick_words, (size_t)2 * KSIM_PICK_WORDS))) return rc;
        h->pick_clear = true;
      }
      // A new geometry: a record slot of a block beyond the last call's grid still holds the tag of
      // some older call, which the 8-bit tags (1..254) can come back to; both buffers are cleared
      // (tag 0 is never used).  Within one geometry every call writes every word its readers read
      // in the record buffer of its parity (pass-A words included), so a word always carries the
      // tag of this call or of the previous call of that parity.
      if (h->pick_clear) {
        HIPCHK(h, hipMemsetAsync(h->pick_words, 0, (size_t)2 * KSIM_PICK_WORDS * 8, ksim_stream(h)));
        h->pick_clear = false;
      }
      h->pick_tag = h->pick_tag % 254u + 1u;
      if (serve_wanted(h) && h->serve_fits && pod->port_cnt <= KSIM_ONE_PORTS && pod->scalar_cnt <= KSIM_MAX_SCALAR) {
        KsimGate gate(h, false);
        // the last SCHEDULE_ONLY was not followed by its AssumePod: undo its tentative commit (this
        // message carries the undo)
        if (h->tent.live && (rc = ksim_tent_undo(h))) return rc;
        if ((rc = serve_ready(h, npt, grid))) return rc;
        oc.lap(0);
        const ksim_pod sp = staged_pod(h, *pod);
        // SCHEDULE_ONLY: a tentative commit, so the AssumePod that normally follows costs no message
        // (KSIM_TENTATIVE=0: decide only).  Not with the service-affinity lender tables: a commit
        // records its label disagreements (ksim_svc_commit), which no undo takes back.
        static const bool tent_off = getenv("KSIM_TENTATIVE") && getenv("KSIM_TENTATIVE")[0] == '0';
        const bool svc = ksim_rt_svc_lender_on(h);
        const int32_t nc = assume ? 0 : (!tent_off && !svc ? KSIM_SERVE_TENTATIVE : 1);
        int32_t r[KSIM_RES_WORDS];
        if ((rc = serve_post(h, KSIM_SERVE_SCHEDULE, sp, ports + pod->port_off, scalars + pod->scalar_off, nc, -1, h->pick_tag,
                             r)))
          return rc;
        oc.lap(2);
        memset(out, 0, sizeof *out);
        out->node = r[KSIM_RES_NODE];
        out->fit_nodes = r[KSIM_RES_FIT];
        memcpy(&out->last_node_index, r + KSIM_RES_CTR, 8);
        if (out->node < 0) memcpy(out->reasons, r + KSIM_RES_REASONS, sizeof out->reasons);
        if (r[KSIM_RES_ERR] & 128) {
          // the refusal clears its flag in the device error word: not under a resident kernel that
          // reads it (the next message relaunches)
          if ((rc = ksim_serve_stop(h))) return rc;
          return ksim_rt_svc_refusal(h);
        }
        if (r[KSIM_RES_ERR] || out->node == INT32_MIN) {
          uint64_t d2[2] = {0, 0};  // the kernel's note of its first failure (site, block, tag, message)
          const int32_t err = r[KSIM_RES_ERR];
          h->serve_off = true;
          if (h->serve_live.load()) (void)ksim_serve_stop(h);
          (void)hipMemcpy(d2, h->ctx.dbg + 96, sizeof d2, hipMemcpyDeviceToHost);
          return ksim_fail(h, KSIM_E_DEVICE, "device consistency error 0x%x (resident pick; site %llu block %llu tag %llu "
                           "message %llu detail 0x%llx; this message %llu tag %u)", err,
                           (unsigned long long)(d2[0] & 255), (unsigned long long)((d2[0] >> 8) & 255),
                           (unsigned long long)((d2[0] >> 16) & 255), (unsigned long long)(d2[0] >> 24),
                           (unsigned long long)d2[1], (unsigned long long)h->serve_seq, h->pick_tag);
        }
        if (assume && out->node >= 0) {
          rc = after_commit(h, pod->port_cnt, r);
          oc.lap(3);
          return rc;
        }
        return KSIM_OK;
      }
      KsimGate gate(h, true);  // the pick kernel's blocks wait on each other
      cs.pick = h->pick_words;
      cs.pick_tag = h->pick_tag;
      h->res_host[KSIM_RES_NODE] = INT32_MIN;
      if ((rc = ksim_rt_check_launch_ctx(h, cs, grid, "ksim_schedule_one"))) return rc;
      oc.lap(0);
      hipError_t ep = ksim_launch_pick(&cs, npt, grid, ksim_rt_aux_on(h) ? 1 : 0, ksim_stream(h));
      if (ep != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "pick launch: %s", hipGetErrorString(ep));
      oc.lap(1);
      HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
      oc.lap(2);
      const int32_t* r = h->res_host;
      memset(out, 0, sizeof *out);
      out->node = r[KSIM_RES_NODE];
      out->fit_nodes = r[KSIM_RES_FIT];
      memcpy(&out->last_node_index, r + KSIM_RES_CTR, 8);
      if (out->node < 0) memcpy(out->reasons, r + KSIM_RES_REASONS, sizeof out->reasons);
      if (r[KSIM_RES_ERR] & 128) return ksim_rt_svc_refusal(h);
      if (r[KSIM_RES_ERR] || out->node == INT32_MIN)
        return ksim_fail(h, KSIM_E_DEVICE, "device consistency error 0x%x (pick)", r[KSIM_RES_ERR]);
      if (assume && out->node >= 0) {
        rc = after_commit(h, pod->port_cnt);
        oc.lap(3);
        return rc;
      }
      return KSIM_OK;
    }
  }
  // InterPodAffinity / SelectorSpread reductions (pass A): fused into the scan behind a grid barrier
  // when the grid is co-resident (one launch), else their own launch first
  const bool ipa = ksim_is_aff_host(h, *pod) &&
                   (c.w[KSIM_W_INTERPOD_AFFINITY] || c.w[KSIM_W_SELECTOR_SPREAD] || ksim_rt_aux_on(h)) && !c.no_prio;
  cs.fuse_a = 0;
  if (ipa && !h->fuse_off) {
    const char* fz = getenv("KSIM_FUSE_A");
    if (h->one_fuse_grid != grid) {
      h->one_fuse_ok = !(fz && fz[0] == '0') && ksim_scan_coresident(npt, 1, grid);
      h->one_fuse_grid = grid;
    }
    cs.fuse_a = h->one_fuse_ok ? 1 : 0;
  }
  h->res_host[KSIM_RES_NODE] = INT32_MIN;  // still there after the wait: the fused barrier gave up
  if ((rc = ksim_rt_check_launch_ctx(h, cs, grid, "ksim_schedule_one"))) return rc;
  KsimGate gate(h, cs.fuse_a != 0);  // the fused pass A: a grid barrier
  hipError_t e = hipSuccess;
  oc.lap(0);
  if (ipa && !cs.fuse_a) e = ksim_launch_ipa_pass(&cs, npt, grid, ksim_stream(h));
  if (e == hipSuccess) e = ksim_launch_scan(&cs, npt, 1, grid, ksim_stream(h));
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "scan launch: %s", hipGetErrorString(e));
  oc.lap(1);
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));  // the result block is host memory: nothing to copy
  oc.lap(2);
  const int32_t* r = h->res_host;
  if (cs.fuse_a && r[KSIM_RES_NODE] == INT32_MIN) {
    // the fused pass-A barrier timed out (blocks not co-resident after all): nothing was decided or
    // committed.  Re-arm the tickets and pass-A scratch and run this pod with pass A as its own launch.
    int32_t err = 0;
    HIPCHK(h, hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
    err &= ~64;
    HIPCHK(h, hipMemcpy(c.err, &err, 4, hipMemcpyHostToDevice));
    HIPCHK(h, hipMemset(c.ticket, 0, 16));
    HIPCHK(h, hipMemset(h->aff_h.ticket, 0, 16));
    if (h->aff_h.n_zone) HIPCHK(h, hipMemset(h->aff_h.zsum, 0, (size_t)h->aff_h.n_zone * 8));
    if (h->aff_h.n_adom) HIPCHK(h, hipMemset(h->aff_h.asum, 0, (size_t)h->aff_h.n_adom * 8));
    h->fuse_off = true;
    return ksim_schedule_one(h, pod, ports, n_ports, scalars, n_scalars, assume, out);
  }
  memset(out, 0, sizeof *out);
  out->node = r[KSIM_RES_NODE];
  out->fit_nodes = r[KSIM_RES_FIT];
  memcpy(&out->last_node_index, r + KSIM_RES_CTR, 8);
  if (out->node < 0) memcpy(out->reasons, r + KSIM_RES_REASONS, sizeof out->reasons);
  if (assume && out->node >= 0) {
    rc = after_commit(h, pod->port_cnt);
    oc.lap(3);
    return rc;
  }
  if (r[KSIM_RES_ERR] & 128) return ksim_rt_svc_refusal(h);
  if (r[KSIM_RES_ERR]) return ksim_fail(h, KSIM_E_DEVICE, "device consistency error 0x%x", r[KSIM_RES_ERR]);
  return KSIM_OK;
}

static int pod_delta(ksim_handle* h, int64_t node, const ksim_pod* pod, const uint64_t* ports, int32_t n_ports,
                     const ksim_scalar_req* scalars, int32_t n_scalars, bool add, const char* where) {
  KsimCtrKeep keep(h);  // (a cache event never moves lastNodeIndex)
  int rc = check_ready(h, where);
  if (rc) return rc;
  if ((rc = check_pod_args(h, pod, n_ports, n_scalars, ports, scalars, where))) return rc;
  if (node < 0 || node >= h->ctx.n) return ksim_fail(h, KSIM_E_INVAL, "%s: node %lld out of range", where, (long long)node);
  // Scheduler.assume after a SCHEDULE_ONLY of this pod onto this node (scheduler.go:366-397,
  // cache.AssumePod cache.go:125-143): the resident kernel committed it tentatively, so it stands
  if (add && h->tent.live && tent_confirms(h, node, *pod, ports, scalars)) {
    h->tent.live = false;
    h->tent.act = KSIM_TENT_CONFIRM;  // (the next message lets the record go)
    h->tent_stats[3] += 1;
    return after_commit(h, pod->port_cnt, h->tent.res);
  }
  if ((rc = ksim_rt_check_aff(h, where))) return rc;
  if (add && (rc = ensure_port_room(h, pod->port_cnt))) return rc;
  ksim_pod p = *pod;
  p.host = -1;  // spec.nodeName plays no part in a resource delta (the node is given)
  if ((rc = ksim_rt_check_pod(h, p, n_ports, n_scalars, scalars, where))) return rc;
  // the resident per-pod kernel takes an assume as a message (the adapter's Schedule + AssumePod
  // pattern), when it serves the current context
  if (add && h->serve_live.load() && p.port_cnt <= KSIM_ONE_PORTS && p.scalar_cnt <= KSIM_MAX_SCALAR) {
    KsimGate gate(h, false);
    if (h->tent.live && (rc = ksim_tent_undo(h))) return rc;
    if (h->serve_live.load() && memcmp(&h->ctx, &h->serve_base, sizeof(KsimCtx)) == 0) {
      int32_t r[KSIM_RES_WORDS];
      if ((rc = serve_post(h, KSIM_SERVE_ASSUME, staged_pod(h, p), ports + p.port_off, scalars + p.scalar_off, 0, node, 0, r)))
        return rc;
      return after_commit(h, pod->port_cnt, r);
    }
  }
  KsimCtx cs;
  if ((rc = stage_pod(h, p, ports, scalars, &cs))) return rc;
  hipError_t e = add ? ksim_launch_assume(&cs, 0, node, h->res_dev + KSIM_RES_STATUS, ksim_stream(h))
                     : ksim_launch_release(&cs, 0, node, ksim_stream(h));
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "%s launch: %s", where, hipGetErrorString(e));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  if (!add) {  // a release can only shrink quantities, but never below zero in a consistent cache
    h->tree_valid = false;
    return KSIM_OK;
  }
  return after_commit(h, pod->port_cnt);
}

int ksim_pod_add(ksim_handle* h, int64_t node, const ksim_pod* pod, const uint64_t* ports, int32_t n_ports,
                 const ksim_scalar_req* scalars, int32_t n_scalars) {
  return pod_delta(h, node, pod, ports, n_ports, scalars, n_scalars, true, "ksim_pod_add");
}

int ksim_pod_remove(ksim_handle* h, int64_t node, const ksim_pod* pod, const uint64_t* ports, int32_t n_ports,
                    const ksim_scalar_req* scalars, int32_t n_scalars) {
  return pod_delta(h, node, pod, ports, n_ports, scalars, n_scalars, false, "ksim_pod_remove");
}

int ksim_assume(ksim_handle* h, int64_t pod, int64_t node) {
  if (!h) return ksim_fail(h, KSIM_E_INVAL, "ksim_assume: null handle");
  if (!h->have_pods) return ksim_fail(h, KSIM_E_STATE, "ksim_assume: nothing loaded");
  if (pod < 0 || pod >= h->n_pods || node < 0 || node >= h->ctx.n) return ksim_fail(h, KSIM_E_INVAL, "ksim_assume: out of range");
  HIPCHK(h, hipSetDevice(h->device));
  int rc = ksim_rt_check_aff(h, "ksim_assume");
  if (rc) return rc;
  rc = ensure_staging(h, 0, 0);
  if (rc) return rc;
  memset(h->res_host, 0, KSIM_RES_WORDS * 4);
  hipError_t e = ksim_launch_assume(&h->ctx, pod, node, h->res_dev + KSIM_RES_STATUS, ksim_stream(h));
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "assume launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  return after_commit(h, 0);
}

int ksim_node_add(ksim_handle* h, int64_t index, const ksim_node_row* row) {
  KsimCtrKeep keep(h);
  int rc = check_ready(h, "ksim_node_add");
  if (rc) return rc;
  if (index < 0 || index > h->ctx.n) return ksim_fail(h, KSIM_E_INVAL, "ksim_node_add: rank %lld out of range", (long long)index);
  if (h->ctx.n >= (int64_t)INT32_MAX) return ksim_fail(h, KSIM_E_INVAL, "ksim_node_add: too many nodes");
  if ((rc = check_row(h, row, true, "ksim_node_add"))) return rc;
  if (row->port_count > h->ctx.port_slots &&
      (rc = grow_port_slots(h, std::max({row->port_count, 2 * h->ctx.port_slots, 4}))))
    return rc;
  if ((rc = node_shift(h, KSIM_RELAY_INSERT, index))) return rc;
  node_event(h);
  if ((rc = set_row(h, index, row, true))) return rc;
  h->port_bound = std::max<int64_t>(h->port_bound, row->port_count);
  h->max_label_set = std::max(h->max_label_set, row->label_set);
  h->max_taint_set = std::max(h->max_taint_set, row->taint_set);
  return KSIM_OK;
}

int ksim_node_update(ksim_handle* h, int64_t index, const ksim_node_row* row) {
  KsimCtrKeep keep(h);
  int rc = check_ready(h, "ksim_node_update");
  if (rc) return rc;
  if (index < 0 || index >= h->ctx.n) return ksim_fail(h, KSIM_E_INVAL, "ksim_node_update: rank %lld out of range", (long long)index);
  if ((rc = check_row(h, row, false, "ksim_node_update"))) return rc;
  if ((rc = set_row(h, index, row, false))) return rc;
  node_event(h);                 // labels may have changed: topology domains
  ksim_rt_invalidate_layout(h);  // allocatable feeds the trees' and sweeps' derived columns
  h->max_label_set = std::max(h->max_label_set, row->label_set);
  h->max_taint_set = std::max(h->max_taint_set, row->taint_set);
  return KSIM_OK;
}

int ksim_node_remove(ksim_handle* h, int64_t index) {
  KsimCtrKeep keep(h);
  int rc = check_ready(h, "ksim_node_remove");
  if (rc) return rc;
  if (index < 0 || index >= h->ctx.n) return ksim_fail(h, KSIM_E_INVAL, "ksim_node_remove: rank %lld out of range", (long long)index);
  node_event(h);
  return node_shift(h, KSIM_RELAY_REMOVE, index);
}

int ksim_node_count(ksim_handle* h, int64_t* out) {
  if (!h || !out) return ksim_fail(h, KSIM_E_INVAL, "ksim_node_count: null argument");
  *out = h->have_nodes ? h->ctx.n : 0;
  return KSIM_OK;
}

}  // extern "C"
