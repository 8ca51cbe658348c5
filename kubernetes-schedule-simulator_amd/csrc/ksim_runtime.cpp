// ksim_runtime.cpp — host side of libksim.so: the C-ABI declared in include/ksim.h.
//
// Owns the device-resident node table (SoA columns in HBM), the pod-class tables, the
// pod queue and the run state, and drives the scan kernels on one HIP stream per handle.
// No torch types cross this boundary; every entry point calls hipSetDevice (cgo calls may
// land on any OS thread) and returns a KSIM_* status.
#include "ksim_handle.h"

namespace {
thread_local std::string g_err;
}  // namespace

int ksim_fail(ksim_handle* h, int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  if (h) h->err = buf;
  g_err = buf;
  return code;
}

extern "C" {

int ksim_abi_version(void) { return KSIM_ABI_VERSION; }

const char* ksim_last_error(const ksim_handle* h) { return h ? h->err.c_str() : g_err.c_str(); }

int ksim_create(const ksim_config* cfg, ksim_handle** out) {
  if (!cfg || !out) return ksim_fail(nullptr, KSIM_E_INVAL, "ksim_create: null argument");
  *out = nullptr;
  int ndev = 0;
  hipError_t e = hipGetDeviceCount(&ndev);
  if (e != hipSuccess || ndev == 0)
    return ksim_fail(nullptr, KSIM_E_DEVICE, "ksim_create: no HIP device (%s)", hipGetErrorString(e));
  if (cfg->device < 0 || cfg->device >= ndev) return ksim_fail(nullptr, KSIM_E_INVAL, "ksim_create: bad device %d", cfg->device);
  for (int k = 0; k < KSIM_NW; ++k)
    if (cfg->weights[k] < 0) return ksim_fail(nullptr, KSIM_E_INVAL, "ksim_create: negative weight in slot %d", k);
  if (cfg->mode < KSIM_MODE_AUTO || cfg->mode > KSIM_MODE_TREE)
    return ksim_fail(nullptr, KSIM_E_INVAL, "ksim_create: unknown mode %d", cfg->mode);
  const uint32_t known = (1u << 19) - 1;  // KSIM_P_CHECK_NODE_CONDITION .. KSIM_P_SERVICE_AFFINITY
  if (cfg->predicates & ~known) return ksim_fail(nullptr, KSIM_E_UNSUPPORTED, "ksim_create: unknown predicate bits");
  ksim_handle* h = new ksim_handle();
  h->device = cfg->device;
  h->cfg = *cfg;
  if (hipSetDevice(h->device) != hipSuccess || hipStreamCreateWithFlags(&h->stream_raw, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreate(&h->ev0) != hipSuccess || hipEventCreate(&h->ev1) != hipSuccess) {
    delete h;
    return ksim_fail(nullptr, KSIM_E_DEVICE, "ksim_create: stream/event creation failed");
  }
  KsimCtx& c = h->ctx;
  c.preds = cfg->predicates;
  c.no_prio = cfg->no_priorities;
  c.collect = cfg->collect_reasons;
  for (int k = 0; k < KSIM_NW; ++k) c.w[k] = cfg->weights[k];
  int rc;
  if ((rc = dev_alloc(h, &c.cursor, 1)) || (rc = dev_alloc(h, &c.counter, 1)) || (rc = dev_alloc(h, &c.ticket, 4)) ||
      (rc = dev_alloc(h, &c.err, 4)) || (rc = dev_alloc(h, &c.dbg, 128))) {
    ksim_destroy(h);
    return rc;
  }
  (void)hipMemsetAsync(c.ticket, 0, 16, ksim_stream(h));
  (void)hipMemsetAsync(c.err, 0, 16, ksim_stream(h));
  (void)hipMemsetAsync(c.dbg, 0, 128 * sizeof(uint64_t), ksim_stream(h));
  (void)hipMemcpyAsync(c.counter, &cfg->last_node_index, 8, hipMemcpyHostToDevice, ksim_stream(h));
  if (hipStreamSynchronize(ksim_stream(h)) != hipSuccess) {
    ksim_destroy(h);
    return ksim_fail(nullptr, KSIM_E_DEVICE, "ksim_create: initial copies failed");
  }
  if (const char* g = getenv("KSIM_MAX_GRID")) h->max_grid = atoi(g);
  // fused pass A's grid-barrier bound: 2 s (KSIM_BARRIER_TICKS, 100 MHz ticks: tests force the bail path)
  c.barrier_ticks = 200000000ull;
  if (const char* b = getenv("KSIM_BARRIER_TICKS")) c.barrier_ticks = strtoull(b, nullptr, 10);
  *out = h;
  return KSIM_OK;
}

void ksim_destroy(ksim_handle* h) {
  if (!h) return;
  (void)hipSetDevice(h->device);
  if (h->stream_raw) (void)hipStreamSynchronize(ksim_stream(h));  // (stops the resident per-pod kernel)
  if (h->serve_live.load()) (void)hipStreamSynchronize(h->stream_raw);  // (its stop failed: let it leave by its idle vote)
  ksim_serve_forget(h);
  if (getenv("KSIM_SERVE_STATS") && h->serve_stats[0])
    fprintf(stderr, "[ksim serve] launches %lld messages %lld stops %lld left-idle %lld untaken-relaunches %lld\n",
            (long long)h->serve_stats[0], (long long)h->serve_stats[1], (long long)h->serve_stats[2],
            (long long)h->serve_stats[3], (long long)h->serve_stats[4]);
  if (getenv("KSIM_SERVE_STATS") && h->tent_stats[0])
    fprintf(stderr, "[ksim tentative] commits %lld undone %lld by-launch %lld confirmed %lld\n", (long long)h->tent_stats[0],
            (long long)h->tent_stats[1], (long long)h->tent_stats[2], (long long)h->tent_stats[3]);
#ifdef KSIM_STAMPS
  if (h->ctx.dbg) {  // the scan kernel's phase stamps (ksim_kernels.hip SSTAMP)
    uint64_t d[64];
    if (hipMemcpy(d, h->ctx.dbg, sizeof d, hipMemcpyDeviceToHost) == hipSuccess && d[61]) {
      const double nb = (double)(d[60] ? d[60] : 1), nl = (double)d[61];
      fprintf(stderr, "[ksim stamps] scan: %llu launches (%llu blocks), thread-0 cycles per block: pod %.0f eval %.0f "
              "masks+stats %.0f partial+ticket %.0f; last block: combine %.0f decide %.0f locate %.0f pick %.0f commit %.0f "
              "results %.0f\n", (unsigned long long)d[61], (unsigned long long)d[60], d[48] / nb, d[49] / nb, d[50] / nb,
              d[51] / nb, d[52] / nl, d[53] / nl, d[54] / nl, d[55] / nl, d[56] / nl, d[57] / nl);
    }
  }
#endif
  for (void*& m : h->ipc_mapped)
    if (m) { (void)hipIpcCloseMemHandle(m); m = nullptr; }
  if (h->shard.xchg) { (void)hipFree(h->shard.xchg); h->shard.xchg = nullptr; }
  if (h->gexec) (void)hipGraphExecDestroy(h->gexec);
  if (h->graph) (void)hipGraphDestroy(h->graph);
  for (auto& b : h->bufs) (void)hipFree(b.p);
  if (h->stg_host) (void)hipHostFree(h->stg_host);  // res_host points into it
  if (h->serve_box) (void)hipHostFree(h->serve_box);
  if (h->cls.mirror) (void)hipHostFree(h->cls.mirror);
  if (h->side_stream) (void)hipStreamDestroy(h->side_stream);
  if (h->ev0) (void)hipEventDestroy(h->ev0);
  if (h->ev1) (void)hipEventDestroy(h->ev1);
  if (h->stream_raw) (void)hipStreamDestroy(h->stream_raw);
  delete h;
}

int ksim_load_nodes(ksim_handle* h, const ksim_node_table* t) {
  if (!h || !t) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_nodes: null argument");
  if (h->have_nodes) return ksim_fail(h, KSIM_E_STATE, "ksim_load_nodes: node table already loaded");
  HIPCHK(h, hipSetDevice(h->device));
  const int64_t n = t->n_nodes;
  if (n < 0) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_nodes: negative node count");
  if (n > (int64_t)INT32_MAX) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_nodes: too many nodes");
  if (t->n_scalar < 0 || t->n_scalar > KSIM_MAX_SCALAR) return ksim_fail(h, KSIM_E_UNSUPPORTED, "n_scalar %d > %d", t->n_scalar, KSIM_MAX_SCALAR);
  if (t->port_slots < 0 || t->port_slots > 4096) return ksim_fail(h, KSIM_E_INVAL, "port_slots out of range");
  if (n && (!t->alloc_cpu || !t->alloc_mem || !t->allowed_pods)) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_nodes: missing column");
  KsimCtx& c = h->ctx;
  c.n = n;
  c.n_scalar = t->n_scalar;
  c.port_slots = t->port_slots;
  // derive the library-maintained over-commit bits
  std::vector<uint32_t> fl(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    uint32_t f = t->flags ? (t->flags[i] & 0xFFu) : 0u;
    const int64_t ag = t->alloc_gpu ? t->alloc_gpu[i] : 0, rg = t->req_gpu ? t->req_gpu[i] : 0;
    const int64_t ae = t->alloc_eph ? t->alloc_eph[i] : 0, re = t->req_eph ? t->req_eph[i] : 0;
    if (ag < rg) f |= KSIM_N_GPU_OVER;
    if (ae < re) f |= KSIM_N_EPH_OVER;
    fl[i] = f;
  }
  if (t->port_count && t->ports) {
    for (int64_t i = 0; i < n; ++i) {
      if (t->port_count[i] < 0 || t->port_count[i] > t->port_slots) return ksim_fail(h, KSIM_E_INVAL, "port_count[%lld] out of range", (long long)i);
      h->port_bound = std::max<int64_t>(h->port_bound, t->port_count[i]);
    }
  }
  h->max_label_set = h->max_taint_set = -1;
  for (int64_t i = 0; i < n; ++i) {
    const int32_t ls = t->label_set ? t->label_set[i] : 0, ts = t->taint_set ? t->taint_set[i] : 0;
    if (ls < 0 || ts < 0) return ksim_fail(h, KSIM_E_INVAL, "node %lld: negative label / taint set id", (long long)i);
    h->max_label_set = std::max(h->max_label_set, ls);
    h->max_taint_set = std::max(h->max_taint_set, ts);
  }
  if (h->have_classes && (h->max_label_set >= h->n_label_sets || h->max_taint_set >= h->n_taint_sets))
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_nodes: label / taint set id beyond the loaded class tables");
  const size_t S = (size_t)t->n_scalar;
  int rc;
  int64_t *ac, *am, *ag, *ae, *as;
  int32_t *ap, *ls, *ts;
  if ((rc = dev_upload(h, &ac, t->alloc_cpu, n)) || (rc = dev_upload(h, &am, t->alloc_mem, n)) ||
      (rc = dev_upload(h, &ag, t->alloc_gpu, n)) || (rc = dev_upload(h, &ae, t->alloc_eph, n)) ||
      (rc = dev_upload(h, &ap, t->allowed_pods, n)) || (rc = dev_upload(h, &c.flags, fl.data(), n)) ||
      (rc = dev_upload(h, &ls, t->label_set, n)) || (rc = dev_upload(h, &ts, t->taint_set, n)) ||
      (rc = dev_upload(h, &as, t->alloc_scalar, S * n)) || (rc = dev_upload(h, &c.req_cpu, t->req_cpu, n)) ||
      (rc = dev_upload(h, &c.req_mem, t->req_mem, n)) || (rc = dev_upload(h, &c.req_gpu, t->req_gpu, n)) ||
      (rc = dev_upload(h, &c.req_eph, t->req_eph, n)) || (rc = dev_upload(h, &c.nz_cpu, t->nz_cpu, n)) ||
      (rc = dev_upload(h, &c.nz_mem, t->nz_mem, n)) || (rc = dev_upload(h, &c.pod_count, t->pod_count, n)) ||
      (rc = dev_upload(h, &c.req_scalar, t->req_scalar, S * n)) ||
      (rc = dev_upload(h, &c.ports, t->ports, (size_t)t->port_slots * n)) ||
      (rc = dev_upload(h, &c.port_count, t->ports ? t->port_count : nullptr, n)))
    return rc;
  c.alloc_cpu = ac; c.alloc_mem = am; c.alloc_gpu = ag; c.alloc_eph = ae; c.alloc_scalar = as;
  c.allowed_pods = ap; c.label_set = ls; c.taint_set = ts;
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  {
    const int64_t lim = (int64_t)1 << 48;
    for (const int64_t* col : {t->alloc_cpu, t->req_cpu, t->nz_cpu, t->alloc_mem, t->req_mem, t->nz_mem})
      for (int64_t i = 0; col && i < n; ++i)
        if (col[i] < 0 || col[i] >= lim) h->pfast_off = true;
  }
  h->have_nodes = true;
  return KSIM_OK;
}

// The class tables live at capacity strides (h->cls, ksim_handle.h): a reload that fits the
// capacities writes only the rows that changed (new pod classes: their rows; new label / taint sets:
// every class's row) through a pinned host mirror, on a side stream when the resident per-pod kernel
// runs (its next message acquires: KSIM_SERVE_SYNC_ACQUIRE), so the table pointers and strides stay
// and the resident kernel keeps running.  A reload beyond the capacities doubles them (one stop).
namespace {
constexpr int32_t one = 1;  // n_tt / n_na when the caller passes none
struct ClsArr {
  const void* src;   // the caller's [C][width] array (null: the default)
  int32_t esz;       // element bytes
  int64_t width;     // elements per class (caller)
  int64_t stride;    // elements per class (device, capacity)
  void** dev;        // the ctx pointer
  int64_t mirror;    // byte offset of this array in the pinned mirror
};
}  // namespace

int ksim_load_classes(ksim_handle* h, const ksim_class_tables* t) {
  if (!h || !t) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_classes: null argument");
  HIPCHK(h, hipSetDevice(h->device));
  if (t->n_classes <= 0 || t->n_label_sets <= 0 || t->n_taint_sets <= 0)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_classes: empty tables");
  // a reload (new pod classes, label sets or taint sets) must still cover everything in use
  if (h->have_nodes && (h->max_label_set >= t->n_label_sets || h->max_taint_set >= t->n_taint_sets))
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_classes: the node table uses label / taint sets beyond the new tables");
  for (int32_t k : h->q_cls)
    if (k >= t->n_classes) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_classes: a queued pod uses class %d beyond the new tables", k);
  const int64_t C = t->n_classes, L = t->n_label_sets, T = t->n_taint_sets;
  const int64_t lw = (L + 31) / 32, tw = (T + 31) / 32;
  // the value rows' width: 16, or wider for classes with more values in one reduce dimension
  const int64_t W = t->val_width ? t->val_width : KSIM_MAX_RCLASS;
  if (W < KSIM_MAX_RCLASS || W > KSIM_MAX_WIDE)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_load_classes: val_width %d outside [%d, %d]", t->val_width, KSIM_MAX_RCLASS,
                     KSIM_MAX_WIDE);
  for (int64_t k = 0; k < C; ++k) {
    const int a = t->n_tt ? t->n_tt[k] : 1, b = t->n_na ? t->n_na[k] : 1;
    if (a < 1 || b < 1 || a > W || b > W)
      return ksim_fail(h, KSIM_E_INVAL, "class %lld: %d x %d reduce classes exceed the value rows (%lld)", (long long)k, a, b,
                       (long long)W);
    if ((int64_t)a * b > KSIM_MAX_WIDE)
      return ksim_fail(h, KSIM_E_UNSUPPORTED, "class %lld: %d x %d reduce classes exceed %d", (long long)k, a, b, KSIM_MAX_WIDE);
  }
  KsimCtx& c = h->ctx;
  auto& cl = h->cls;
  const bool has_na = t->na_add != nullptr, has_sv = t->svc_ok != nullptr;
  const bool fits = cl.mirror && C <= cl.cap_c && L <= cl.cap_l && T <= cl.cap_t && has_na == cl.has_na && has_sv == cl.has_sv &&
                    W == cl.w;
  // the row range to write: new classes only, unless the label / taint sets changed (every row)
  int64_t from = fits && L == cl.l && T == cl.t ? std::min<int64_t>(cl.c, C) : 0;
  if (!fits) {
    // (re)allocate at capacity: exact on the first load (batch runs), doubled on growth
    const bool grow = cl.mirror != nullptr;
    const int64_t cc = grow ? std::max<int64_t>(C, 2 * cl.cap_c) : C;
    const int64_t cL = grow ? std::max<int64_t>(L, L > cl.cap_l ? 2 * cl.cap_l : cl.cap_l) : L;
    const int64_t cT = grow ? std::max<int64_t>(T, T > cl.cap_t ? 2 * cl.cap_t : cl.cap_t) : T;
    HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));  // (stops the resident kernel: new pointers)
    for (void* q : h->class_bufs) dev_free(h, q);
    h->class_bufs.clear();
    if (cl.mirror) { (void)hipHostFree(cl.mirror); cl.mirror = nullptr; }
    c.sel_ok = c.taint_ok = c.noexec_ok = c.svc_ok = nullptr;
    c.tt_class = c.na_class = nullptr;
    c.n_tt = c.n_na = nullptr;
    c.tt_val = c.na_val = c.na_add = nullptr;
    cl.cap_c = cc; cl.cap_l = cL; cl.cap_t = cT;
    cl.w = W;
    cl.has_na = has_na; cl.has_sv = has_sv;
  }
  const int64_t lwc = (cl.cap_l + 31) / 32, twc = (cl.cap_t + 31) / 32;
  ClsArr arr[] = {
      {t->sel_ok, 4, lw, lwc, (void**)&c.sel_ok, 0},      {t->taint_ok, 4, tw, twc, (void**)&c.taint_ok, 0},
      {t->noexec_ok, 4, tw, twc, (void**)&c.noexec_ok, 0}, {t->tt_class, 1, T, cl.cap_t, (void**)&c.tt_class, 0},
      {t->na_class, 1, L, cl.cap_l, (void**)&c.na_class, 0}, {t->n_tt, 4, 1, 1, (void**)&c.n_tt, 0},
      {t->n_na, 4, 1, 1, (void**)&c.n_na, 0},              {t->tt_val, 8, W, W, (void**)&c.tt_val, 0},
      {t->na_val, 8, W, W, (void**)&c.na_val, 0},
      {t->na_add, 8, W, W, (void**)&c.na_add, 0},
      {t->svc_ok, 4, lw, lwc, (void**)&c.svc_ok, 0}};
  const int n_arr = 9 + (has_na ? 1 : 0) + (has_sv ? 1 : 0);
  if (!has_na) arr[9] = arr[10];  // (the optional arrays compacted to the end)
  int64_t mb = 0;
  for (int k = 0; k < n_arr; ++k) {
    arr[k].mirror = mb;
    mb += (cl.cap_c * arr[k].stride * arr[k].esz + 255) / 256 * 256;
  }
  if (!cl.mirror) {
    HIPCHK(h, hipHostMalloc((void**)&cl.mirror, (size_t)mb, hipHostMallocDefault));
    memset(cl.mirror, 0, (size_t)mb);
    const size_t nb0 = h->bufs.size();
    for (int k = 0; k < n_arr; ++k) {
      char* q = nullptr;
      int rc = dev_alloc(h, &q, (size_t)(cl.cap_c * arr[k].stride * arr[k].esz));
      if (rc) return rc;
      *arr[k].dev = q;
    }
    for (size_t k = nb0; k < h->bufs.size(); ++k) h->class_bufs.push_back(h->bufs[k].p);
  }
  // "A superset" is not trusted row by row: the first row any array changes (callers rebuild their
  // tables, and a placeholder row may be filled in later) moves `from` back
  for (int k = 0; k < n_arr && from > 0; ++k) {
    const ClsArr& x = arr[k];
    const size_t rb = (size_t)(x.width * x.esz), sb = (size_t)(x.stride * x.esz);
    const char* m = cl.mirror + x.mirror;
    for (int64_t r = 0; r < from; ++r) {
      const char* src = static_cast<const char*>(x.src) + (size_t)r * rb;
      const bool same = x.src ? memcmp(m + (size_t)r * sb, src, rb) == 0
                              : (x.esz == 4 && x.width == 1 ? memcmp(m + (size_t)r * sb, &one, 4) == 0 : true);
      if (!same) { from = r; break; }
    }
  }
  // rows [from, C) into the mirror at capacity strides, then to the device
  for (int k = 0; k < n_arr; ++k) {
    const ClsArr& x = arr[k];
    char* m = cl.mirror + x.mirror;
    const size_t rb = (size_t)(x.width * x.esz), sb = (size_t)(x.stride * x.esz);
    for (int64_t r = from; r < C; ++r) {
      char* d = m + (size_t)r * sb;
      if (x.src) memcpy(d, static_cast<const char*>(x.src) + (size_t)r * rb, rb);
      else if (x.esz == 4 && x.width == 1) memcpy(d, &one, 4);  // n_tt / n_na default 1
      else memset(d, 0, rb);
      if (sb > rb) memset(d + rb, 0, sb - rb);
    }
  }
  // the resident per-pod kernel keeps running when the pointers stay: the rows go on a side stream
  // (it reads no class row between messages) and its next message acquires them
  const bool side = fits && h->serve_live.load();
  if (side && !h->side_stream) HIPCHK(h, hipStreamCreateWithFlags(&h->side_stream, hipStreamNonBlocking));
  hipStream_t st = side ? h->side_stream : ksim_stream(h);
  if (C > from)
    for (int k = 0; k < n_arr; ++k) {
      const ClsArr& x = arr[k];
      const size_t sb = (size_t)(x.stride * x.esz);
      HIPCHK(h, hipMemcpyAsync(static_cast<char*>(*x.dev) + (size_t)from * sb, cl.mirror + x.mirror + (size_t)from * sb,
                               (size_t)(C - from) * sb, hipMemcpyHostToDevice, st));
    }
  HIPCHK(h, hipStreamSynchronize(st));
  if (side) h->serve_shared = true;  // (the next message acquires the new rows)
  cl.c = C; cl.l = L; cl.t = T;
  cl.loads += 1;
  cl.in_place += side ? 1 : 0;
  if (!has_na) c.na_add = nullptr;
  if (!has_sv) c.svc_ok = nullptr;
  c.use_na = (c.w[KSIM_W_NODE_AFFINITY] != 0 || has_na) ? 1 : 0;
  // strides are the capacities (every kernel indexes [class * stride + column])
  c.lwords = (int32_t)lwc; c.twords = (int32_t)twc;
  c.n_label_sets = (int32_t)cl.cap_l; c.n_taint_sets = (int32_t)cl.cap_t;
  c.n_classes_dev = (int32_t)C;
  c.val_w = (int32_t)W;
  // the resident kernel reads no class count (only rows through the strides above, which stayed)
  if (side) h->serve_base.n_classes_dev = c.n_classes_dev;
  h->n_classes = t->n_classes;
  h->n_label_sets = t->n_label_sets;
  h->n_taint_sets = t->n_taint_sets;
  const int32_t* ntt = t->n_tt, *nna = t->n_na;
  h->h_n_tt.resize(C);
  h->h_n_na.resize(C);
  for (int64_t k = 0; k < C; ++k) {
    h->h_n_tt[k] = ntt ? ntt[k] : 1;
    h->h_n_na[k] = nna ? nna[k] : 1;
  }
  h->any_wide = false;
  for (int64_t k = 0; k < C; ++k) h->any_wide |= wide_k(h, (int32_t)k);
  // class pointers are baked into the launch graph's kernel arguments
  if (!fits) {
    if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
    if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
  }
  if (h->have_classes) ksim_rt_recompute_fast(h);  // reduce-class counts decide fast-kernel eligibility
  if (h->n_pods) {  // and ride in the queued descriptors (ksim_persistent.hip's ring)
    hipError_t e = ksim_launch_pod_k(h->d_pods, h->n_pods, &c, ksim_stream(h));
    if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "pod k launch: %s", hipGetErrorString(e));
    HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  }
  h->have_classes = true;
  return KSIM_OK;
}

int ksim_load_pods(ksim_handle* h, const ksim_pod* pods, int64_t n_pods, const uint64_t* ports, int64_t n_ports,
                   const ksim_scalar_req* scalars, int64_t n_scalars) {
  if (!h || (!pods && n_pods)) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_pods: null argument");
  if (!h->have_nodes || !h->have_classes) return ksim_fail(h, KSIM_E_STATE, "ksim_load_pods: load nodes and classes first");
  if (h->have_pods) return ksim_fail(h, KSIM_E_STATE, "ksim_load_pods: pod queue already loaded (use ksim_append_pods)");
  return ksim_rt_append(h, pods, n_pods, ports, n_ports, scalars, n_scalars);
}

int ksim_append_pods(ksim_handle* h, const ksim_pod* pods, int64_t n_pods, const uint64_t* ports, int64_t n_ports,
                     const ksim_scalar_req* scalars, int64_t n_scalars) {
  if (!h || (!pods && n_pods)) return ksim_fail(h, KSIM_E_INVAL, "ksim_append_pods: null argument");
  if (!h->have_nodes || !h->have_classes) return ksim_fail(h, KSIM_E_STATE, "ksim_append_pods: load nodes and classes first");
  return ksim_rt_append(h, pods, n_pods, ports, n_ports, scalars, n_scalars);
}

}  // extern "C"

int ksim_rt_check_pod(ksim_handle* h, const ksim_pod& p, int64_t n_ports, int64_t n_scalars,
                      const ksim_scalar_req* scalars, const char* where) {
  const KsimCtx& c = h->ctx;
  if (p.cls < 0 || p.cls >= h->n_classes) return ksim_fail(h, KSIM_E_INVAL, "%s: class %d out of range", where, p.cls);
  if (p.host < -2 || p.host >= c.n) return ksim_fail(h, KSIM_E_INVAL, "%s: host %d out of range", where, p.host);
  if (p.port_cnt < 0 || p.port_off < 0 || (int64_t)p.port_off + p.port_cnt > n_ports)
    return ksim_fail(h, KSIM_E_INVAL, "%s: port range out of bounds", where);
  if (p.scalar_cnt < 0 || p.scalar_off < 0 || (int64_t)p.scalar_off + p.scalar_cnt > n_scalars)
    return ksim_fail(h, KSIM_E_INVAL, "%s: scalar range out of bounds", where);
  if (p.port_cnt > 0 && c.port_slots == 0)
    return ksim_fail(h, KSIM_E_INVAL, "%s requests host ports but the node table has no port slots", where);
  for (int32_t s = 0; s < p.scalar_cnt; ++s)
    if (scalars[p.scalar_off + s].col < 0 || scalars[p.scalar_off + s].col >= c.n_scalar)
      return ksim_fail(h, KSIM_E_INVAL, "%s: scalar request column out of range", where);
  if ((p.aff_ident || p.aff_class) && !h->have_aff)
    return ksim_fail(h, KSIM_E_STATE, "%s: affinity identity / class set but no affinity tables are loaded", where);
  if (p.aff_ident < 0 || p.aff_ident > h->aff_n_ident || p.aff_class < 0 || p.aff_class > h->aff_n_aclass)
    return ksim_fail(h, KSIM_E_INVAL, "%s: affinity identity / class out of range", where);
  if (p.vol_class && !h->have_vol)
    return ksim_fail(h, KSIM_E_STATE, "%s: volume class set but no volume tables are loaded", where);
  if (p.vol_class < 0 || p.vol_class > h->vol_n_class)
    return ksim_fail(h, KSIM_E_INVAL, "%s: volume class out of range", where);
  return KSIM_OK;
}

int64_t ksim_rt_aff_count(const ksim_handle* h, int64_t first, int64_t count) {
  if (!h->have_aff || count <= 0) return 0;
  return h->aff_pre[first + count] - h->aff_pre[first];
}

int64_t ksim_rt_launch_only_count(const ksim_handle* h, int64_t first, int64_t count) {
  int64_t k = ksim_rt_aff_count(h, first, count);
  if (count > 0) k += h->vol_pre[first + count] - h->vol_pre[first];  // volume and service-affinity pods
  return k;
}

int ksim_rt_svc_refusal(ksim_handle* h) {
  int32_t err = 0;
  HIPCHK(h, hipMemcpy(&err, h->ctx.err, 4, hipMemcpyDeviceToHost));
  err &= ~128;  // the refusal is this call's: the handle stays usable
  HIPCHK(h, hipMemcpy(h->ctx.err, &err, 4, hipMemcpyHostToDevice));
  return ksim_fail(h, KSIM_E_UNSUPPORTED, "CheckServiceAffinity: the cached pods with a pod's labels sit on nodes that disagree "
                                      "on a service-affinity label the pod's nodeSelector leaves open (the pod lister's "
                                      "order would decide)");
}

int ksim_rt_check_aff(ksim_handle* h, const char* where) {
  if (h->have_aff && h->aff_stale)
    return ksim_fail(h, KSIM_E_STATE, "%s: the affinity tables predate a node event; load them again", where);
  if (h->have_vol && h->vol_stale)
    return ksim_fail(h, KSIM_E_STATE, "%s: the volume tables predate a node event; load them again", where);
  return KSIM_OK;
}

// Fast-kernel eligibility of a pod apart from its reduce classes (ksim_is_fast_pod, ksim_fast.h).
static bool fast_base(const ksim_pod& p) {
  const int64_t lim = (int64_t)1 << 48;
  bool in_range = true;
  for (int64_t v : {p.req_cpu, p.req_mem, p.add_cpu, p.add_mem, p.nz_cpu, p.nz_mem}) in_range &= v >= 0 && v < lim;
  return in_range && p.host == -1 && p.port_cnt == 0 && p.scalar_cnt == 0 && p.req_gpu == 0 && p.req_eph == 0 &&
         !(p.flags & (KSIM_POD_NEED_SELECTOR | KSIM_POD_NEED_TAINTS | KSIM_POD_NEED_SVC_AFFINITY)) && p.aff_ident == 0 &&
         p.aff_class == 0 && p.vol_class == 0;
}

static bool fast_k(const ksim_handle* h, int32_t cls) {
  const int k1 = h->ctx.w[KSIM_W_TAINT_TOLERATION] ? h->h_n_tt[cls] : 1;
  const int k2 = h->ctx.use_na ? h->h_n_na[cls] : 1;
  return k1 * k2 == 1;
}

// A pod class with more than KSIM_MAX_RCLASS reduce classes: the launch form's wide decision.
bool wide_k(const ksim_handle* h, int32_t cls) {
  const int k1 = h->ctx.w[KSIM_W_TAINT_TOLERATION] ? h->h_n_tt[cls] : 1;
  const int k2 = h->ctx.use_na ? h->h_n_na[cls] : 1;
  return k1 * k2 > KSIM_MAX_RCLASS;
}

bool ksim_rt_range_wide(const ksim_handle* h, int64_t first, int64_t count) {
  if (!h->any_wide) return false;
  for (int64_t q = first; q < first + count; ++q)
    if (wide_k(h, h->q_cls[q])) return true;
  return false;
}

void ksim_rt_recompute_fast(ksim_handle* h) {
  const int64_t n = (int64_t)h->q_cls.size();
  h->fast_pre.assign((size_t)n + 1, 0);
  for (int64_t i = 0; i < n; ++i)
    h->fast_pre[i + 1] = h->fast_pre[i] + ((h->q_base[i] && fast_k(h, h->q_cls[i])) ? 1 : 0);
}

int ksim_rt_append(ksim_handle* h, const ksim_pod* pods, int64_t n_pods, const uint64_t* ports, int64_t n_ports,
                   const ksim_scalar_req* scalars, int64_t n_scalars) {
  if (n_pods < 0 || n_ports < 0 || n_scalars < 0) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_pods: negative size");
  if ((n_ports && !ports) || (n_scalars && !scalars)) return ksim_fail(h, KSIM_E_INVAL, "ksim_load_pods: null array");
  HIPCHK(h, hipSetDevice(h->device));
  KsimCtx& c = h->ctx;
  char where[64];
  for (int64_t i = 0; i < n_pods; ++i) {
    snprintf(where, sizeof where, "pod %lld", (long long)(h->n_pods + i));
    int rc = ksim_rt_check_pod(h, pods[i], n_ports, n_scalars, scalars, where);
    if (rc) return rc;
  }
  if (h->n_pods + n_pods > (int64_t)INT32_MAX * 8) return ksim_fail(h, KSIM_E_INVAL, "pod queue too long");
  const int64_t P0 = h->n_pods, np = P0 + n_pods;
  const int64_t K0 = h->n_port_keys, S0 = h->n_scalar_reqs;
  if (K0 + n_ports > INT32_MAX || S0 + n_scalars > INT32_MAX) return ksim_fail(h, KSIM_E_INVAL, "pod port / scalar arrays too long");
  int rc;
  // grow the device arrays geometrically (appends amortised); the first load is exact
  auto cap_for = [&](int64_t have, int64_t need) { return have == 0 ? std::max<int64_t>(need, 1) : std::max(need, 2 * have); };
  if (np > h->pod_cap) {
    const int64_t cap = cap_for(h->pod_cap, np);
    int32_t* on = c.out_node;
    if ((rc = dev_grow(h, &h->d_pods, (size_t)P0, (size_t)cap)) || (rc = dev_grow(h, &on, (size_t)P0, (size_t)cap)))
      return rc;
    c.out_node = on;
    if (c.collect) {
      int32_t* orr = c.out_reasons;
      if ((rc = dev_grow(h, &orr, (size_t)P0 * KSIM_NREASONS, (size_t)cap * KSIM_NREASONS))) return rc;
      HIPCHK(h, hipMemsetAsync(orr + P0 * KSIM_NREASONS, 0, (size_t)(cap - P0) * KSIM_NREASONS * 4, ksim_stream(h)));
      c.out_reasons = orr;
    } else if (!c.out_reasons) {
      int32_t* orr;
      if ((rc = dev_alloc(h, &orr, 1))) return rc;
      c.out_reasons = orr;
    }
    h->pod_cap = cap;
  }
  if (K0 + n_ports > h->port_key_cap) {
    const int64_t cap = cap_for(h->port_key_cap, K0 + n_ports);
    if ((rc = dev_grow(h, &h->d_pod_ports, (size_t)K0, (size_t)cap))) return rc;
    h->port_key_cap = cap;
  }
  if (S0 + n_scalars > h->scalar_req_cap) {
    const int64_t cap = cap_for(h->scalar_req_cap, S0 + n_scalars);
    if ((rc = dev_grow(h, &h->d_pod_scalars, (size_t)S0, (size_t)cap))) return rc;
    h->scalar_req_cap = cap;
  }
  // the queue's port / scalar offsets are relative to the passed arrays: rebase them
  std::vector<ksim_pod> v(pods, pods + n_pods);
  for (auto& p : v) {
    p.port_off += (int32_t)K0;
    p.scalar_off += (int32_t)S0;
  }
  if (n_pods) HIPCHK(h, hipMemcpyAsync(h->d_pods + P0, v.data(), n_pods * sizeof(ksim_pod), hipMemcpyHostToDevice, ksim_stream(h)));
  if (n_ports) HIPCHK(h, hipMemcpyAsync(h->d_pod_ports + K0, ports, n_ports * 8, hipMemcpyHostToDevice, ksim_stream(h)));
  if (n_scalars)
    HIPCHK(h, hipMemcpyAsync(h->d_pod_scalars + S0, scalars, n_scalars * sizeof(ksim_scalar_req), hipMemcpyHostToDevice, ksim_stream(h)));
  c.pods = h->d_pods; c.pod_ports = h->d_pod_ports; c.pod_scalars = h->d_pod_scalars;
  {
    hipError_t e = ksim_launch_pod_k(h->d_pods + P0, n_pods, &c, ksim_stream(h));
    if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "pod k launch: %s", hipGetErrorString(e));
  }
  // host bookkeeping: fast-kernel eligibility, tree classes, float64 bounds
  h->q_cls.resize((size_t)np);
  h->q_base.resize((size_t)np);
  h->q_ident.resize((size_t)np);
  h->q_aclass.resize((size_t)np);
  h->aff_pre.resize((size_t)np + 1);
  h->q_vclass.resize((size_t)np);
  h->vol_pre.resize((size_t)np + 1);
  h->fast_pre.resize((size_t)np + 1);
  h->pod_qmax.resize((size_t)np);
  std::vector<int32_t> tc((size_t)n_pods, -1);
  const int32_t ntc0 = h->n_tcls;
  for (int64_t i = 0; i < n_pods; ++i) {
    const ksim_pod& p = pods[i];
    const int64_t q = P0 + i;
    h->q_cls[q] = p.cls;
    h->q_base[q] = fast_base(p) ? 1 : 0;
    h->q_ident[q] = p.aff_ident;
    h->q_aclass[q] = p.aff_class;
    h->aff_pre[q + 1] = h->aff_pre[q] + ((p.aff_ident || p.aff_class) ? 1 : 0);
    h->q_vclass[q] = p.vol_class;
    h->q_max_port = std::max(h->q_max_port, p.port_cnt);
    h->q_max_scal = std::max(h->q_max_scal, p.scalar_cnt);
    h->vol_pre[q + 1] = h->vol_pre[q] + ((p.vol_class || (p.flags & KSIM_POD_NEED_SVC_AFFINITY)) ? 1 : 0);
    const bool fast = h->q_base[q] && fast_k(h, p.cls);
    h->fast_pre[q + 1] = h->fast_pre[q] + (fast ? 1 : 0);
    int64_t m = 0;
    for (int64_t x : {p.req_cpu, p.req_mem, p.add_cpu, p.add_mem, p.nz_cpu, p.nz_mem}) m = std::max(m, x);
    h->pod_qmax[q] = m;
    // tree class: resource-only pods with identical predicate / priority inputs
    if (!fast || h->n_tcls < 0) continue;
    const std::array<int64_t, 5> key{p.req_cpu, p.req_mem, p.nz_cpu, p.nz_mem,
                                     (int64_t)(p.flags & (KSIM_POD_ANY_REQUEST | KSIM_POD_BEST_EFFORT))};
    auto it = h->tkeys.find(key);
    int32_t k = it == h->tkeys.end() ? (int32_t)h->tkeys.size() : it->second;
    if (it == h->tkeys.end()) {
      if (k == KSIM_TREE_MAX_CLASSES) { h->n_tcls = -1; continue; }
      h->tkeys.emplace(key, k);
      h->tclass_h.push_back(KsimTreeClass{(double)p.req_cpu, (double)p.req_mem, (double)p.nz_cpu, (double)p.nz_mem,
                                          (p.flags & KSIM_POD_ANY_REQUEST) ? ~0u : 0u,
                                          (p.flags & KSIM_POD_BEST_EFFORT) ? ~0u : 0u});
    }
    tc[i] = k;
  }
  if (h->n_tcls >= 0) {
    if (np > h->tcls_cap) {
      const int64_t cap = cap_for(h->tcls_cap, np);
      if ((rc = dev_grow(h, &h->tcls, (size_t)P0, (size_t)cap))) return rc;
      h->tcls_cap = cap;
    }
    if (n_pods) HIPCHK(h, hipMemcpyAsync(h->tcls + P0, tc.data(), n_pods * 4, hipMemcpyHostToDevice, ksim_stream(h)));
    const int32_t ntc = (int32_t)h->tkeys.size();
    if (ntc != ntc0 || !h->tclass) {  // new classes: re-upload the inputs, re-plan the trees
      if (h->tclass) dev_free(h, h->tclass);
      h->tclass = nullptr;
      if ((rc = dev_upload(h, &h->tclass, h->tclass_h.data(), h->tclass_h.size()))) return rc;
      if (ntc != ntc0 && h->tree_planned) {
        for (void* q : {(void*)h->t_leaves, (void*)h->t_levels, (void*)h->t_fit}) dev_free(h, q);
        h->t_leaves = nullptr; h->t_levels = nullptr; h->t_fit = nullptr;
        h->tree_planned = h->tree_ok = h->tree_valid = false;
      }
      h->n_tcls = ntc;
    }
  } else if (h->tree_planned) {
    h->tree_ok = h->tree_valid = false;
  }
  h->n_pods = np;
  h->n_port_keys = K0 + n_ports;
  h->n_scalar_reqs = S0 + n_scalars;
  // queue pointers are baked into the launch graph's kernel arguments
  if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
  if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  h->have_pods = true;
  return KSIM_OK;
}

int ksim_rt_pick_npt(int64_t n) {
  for (int npt : {1, 2, 4, 8})
    if ((n + (int64_t)KSIM_BLOCK * npt - 1) / ((int64_t)KSIM_BLOCK * npt) <= 1024) return npt;
  return 8;
}

int ksim_rt_ensure_partials(ksim_handle* h, int grid) {
  KsimCtx& c = h->ctx;
  if (c.partials && h->part_cap >= grid) return KSIM_OK;
  KsimPartial* p;
  uint64_t* pm;
  int64_t* wm;
  int32_t* wc;
  const size_t cap = (size_t)std::max(grid, 1024);
  int rc = dev_alloc(h, &p, cap);
  if (rc) return rc;
  if ((rc = dev_alloc(h, &pm, cap * KSIM_PM_STRIDE))) { dev_free(h, p); return rc; }
  if ((rc = dev_alloc(h, &wm, cap * KSIM_MAX_WIDE)) || (rc = dev_alloc(h, &wc, cap * KSIM_MAX_WIDE))) return rc;
  dev_free(h, c.partials);
  dev_free(h, c.pmask);
  dev_free(h, c.wmx);
  dev_free(h, c.wcnt);
  c.partials = p;
  c.pmask = pm;
  c.wmx = wm;
  c.wcnt = wc;
  h->part_cap = std::max(grid, 1024);
  if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
  if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
  return KSIM_OK;
}

// Before a launch-form kernel runs on a context: every scratch pointer it may read or write is
// set and sized for the grid (a stale copy of the handle's context would fault on the device).
int ksim_rt_check_launch_ctx(ksim_handle* h, const KsimCtx& c, int grid, const char* where) {
  const void* need[] = {c.partials, c.pmask, c.wmx, c.wcnt, c.ticket, c.err, c.counter, c.cursor, c.pods, c.out_node,
                        c.out_reasons, c.alloc_cpu, c.req_cpu, c.pod_count, c.flags};
  for (const void* p : need)
    if (!p) return ksim_fail(h, KSIM_E_DEVICE, "%s: launch context has an unset scratch / table pointer", where);
  if (grid > h->part_cap) return ksim_fail(h, KSIM_E_DEVICE, "%s: grid %d beyond the partials (%lld)", where, grid,
                                           (long long)h->part_cap);
  if (c.partials != h->ctx.partials || c.pmask != h->ctx.pmask || c.wmx != h->ctx.wmx || c.wcnt != h->ctx.wcnt)
    return ksim_fail(h, KSIM_E_DEVICE, "%s: launch context holds stale scratch pointers", where);
  return KSIM_OK;
}

static int run_launch_mode(ksim_handle* h, int64_t first, int64_t count, ksim_stats* st) {
  KsimCtx& c = h->ctx;
  const int npt = ksim_rt_pick_npt(c.n);
  c.chunk = (int64_t)KSIM_BLOCK * npt;
  const int grid = (int)((c.n + c.chunk - 1) / c.chunk);
  int rc = ksim_rt_ensure_partials(h, grid);
  if (rc) return rc;
  c.first = first;
  c.end = first + count;
  HIPCHK(h, hipMemcpyAsync(c.cursor, &first, 8, hipMemcpyHostToDevice, ksim_stream(h)));
  HIPCHK(h, hipMemsetAsync(c.ticket, 0, 16, ksim_stream(h)));
  const int batch = (int)std::min<int64_t>(count, 256);
  const int ipa = ksim_rt_aff_count(h, first, count) > 0 &&
                  (c.w[KSIM_W_INTERPOD_AFFINITY] != 0 || c.w[KSIM_W_SELECTOR_SPREAD] != 0 || ksim_rt_aux_on(h)) &&
                  !c.no_prio ? 1 : 0;
  // pass A fused into the scan behind a grid barrier when the grid is co-resident (KSIM_FUSE_A=0: two launches)
  const char* fz = getenv("KSIM_FUSE_A");
  // (never node-sharded: pass A's last block waits for the peers, longer than the grid barrier's bound)
  c.fuse_a = ipa && !h->fuse_off && c.sh_world <= 1 && !(fz && fz[0] == '0') && ksim_scan_coresident(npt, c.collect, grid)
                 ? 1 : 0;
  const int gkey = ipa | c.fuse_a << 1;
  if (!h->gexec || h->g_batch != batch || h->g_npt != npt || h->g_collect != c.collect || h->g_first != first ||
      h->g_end != c.end || h->g_ipa != gkey) {
    if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
    if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
    HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
    HIPCHK(h, hipStreamBeginCapture(ksim_stream(h), hipStreamCaptureModeThreadLocal));
    for (int k = 0; k < batch; ++k) {
      hipError_t e = ipa && !c.fuse_a ? ksim_launch_ipa_pass(&c, npt, grid, ksim_stream(h)) : hipSuccess;
      if (e == hipSuccess) e = ksim_launch_scan(&c, npt, c.collect, grid, ksim_stream(h));
      if (e != hipSuccess) {
        hipGraph_t g = nullptr;
        (void)hipStreamEndCapture(ksim_stream(h), &g);
        if (g) (void)hipGraphDestroy(g);
        return ksim_fail(h, KSIM_E_DEVICE, "scan launch during capture: %s", hipGetErrorString(e));
      }
    }
    HIPCHK(h, hipStreamEndCapture(ksim_stream(h), &h->graph));
    HIPCHK(h, hipGraphInstantiate(&h->gexec, h->graph, nullptr, nullptr, 0));
    h->g_batch = batch; h->g_npt = npt; h->g_collect = c.collect; h->g_first = first; h->g_end = c.end; h->g_ipa = gkey;
  }
  const int64_t reps = (count + batch - 1) / batch;
  HIPCHK(h, hipEventRecord(h->ev0, ksim_stream(h)));
  for (int64_t r = 0; r < reps; ++r) HIPCHK(h, hipGraphLaunch(h->gexec, ksim_stream(h)));
  HIPCHK(h, hipEventRecord(h->ev1, ksim_stream(h)));
  HIPCHK(h, hipEventSynchronize(h->ev1));
  float ms = 0.f;
  HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
  if (st) {
    st->device_ms = ms;
    st->kernel_ms = ms;
    st->kernel_launches = reps * batch;
    st->mode = KSIM_MODE_LAUNCH;
    st->blocks = grid;
  }
  if (c.fuse_a) {
    int32_t err = 0;
    HIPCHK(h, hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
    if (err & 64) {
      // the fused pass-A barrier timed out (blocks not co-resident after all, e.g. another handle's
      // kernels on the device): the pod at the cursor was not committed, later launches exited at
      // once.  Re-arm the tickets and pass-A scratch, and finish the range with pass A as its own launch.
      int64_t cur = 0;
      HIPCHK(h, hipMemcpy(&cur, c.cursor, 8, hipMemcpyDeviceToHost));
      err &= ~64;
      HIPCHK(h, hipMemcpy(c.err, &err, 4, hipMemcpyHostToDevice));
      HIPCHK(h, hipMemset(c.ticket, 0, 16));
      HIPCHK(h, hipMemset(h->aff_h.ticket, 0, 16));
      if (h->aff_h.n_zone) HIPCHK(h, hipMemset(h->aff_h.zsum, 0, (size_t)h->aff_h.n_zone * 8));
      if (h->aff_h.n_adom) HIPCHK(h, hipMemset(h->aff_h.asum, 0, (size_t)h->aff_h.n_adom * 8));
      h->fuse_off = true;
      if (cur < first + count) {
        ksim_stats s2{};
        const int rc2 = run_launch_mode(h, cur, first + count - cur, &s2);
        if (rc2) return rc2;
        if (st) {
          st->device_ms += s2.device_ms;
          st->kernel_ms += s2.kernel_ms;
          st->kernel_launches += s2.kernel_launches;
        }
      }
    }
  }
  return KSIM_OK;
}

// Scores travel as 48-bit granule payloads in persistent mode: bound the weights.
static bool persistent_weights_ok(const KsimCtx& c) {
  // map scores are packed into 27 bits of the per-row LDS entry: sum of map weights x
  // MaxPriority < 2^27
  int64_t s = 0;
  for (int k : {KSIM_W_LEAST_REQUESTED, KSIM_W_MOST_REQUESTED, KSIM_W_BALANCED}) {
    if (c.w[k] > ((int64_t)1 << 30)) return false;
    s += c.w[k] * 10;
  }
  return s < ((int64_t)1 << 27);
}

// Form of the specialised kernel (ksim_pfast.hip) for [first, first+count): 0 = not
// applicable (a pod is not resource-only, weights or quantities out of its range), 1 = rows in
// LDS, 2 = rows streamed from HBM (tables beyond the LDS budget, KSIM_FORCE_STREAM for tests).
static int pfast_form(ksim_handle* h, int64_t first, int64_t count, int* grid, int* lds_rows) {
  const KsimCtx& c = h->ctx;
  if (getenv("KSIM_NO_PFAST") || count <= 0 || h->pfast_off || h->fast_pre[first + count] - h->fast_pre[first] != count ||
      !persistent_weights_ok(c))
    return 0;
  if (!getenv("KSIM_FORCE_STREAM") && ksim_pfast_config(c.n, h->max_grid, 0, grid, lds_rows)) return 1;
  if (ksim_pfast_config(c.n, h->max_grid, 1, grid, lds_rows)) return 2;
  return 0;
}

static int run_persistent_mode(ksim_handle* h, int64_t first, int64_t count, ksim_stats* st);

// All pods of [first, first+count) resource-only: the specialised kernel (ksim_pfast.hip).
static int run_pfast_mode(ksim_handle* h, int64_t first, int64_t count, int grid, int lds_rows, bool stream,
                          ksim_stats* st) {
  KsimCtx& c = h->ctx;
  if (stream) {
    if (!h->mirror) {
      int rc = dev_alloc(h, &h->mirror, (size_t)6 * c.n);
      if (rc) return rc;
    }
    hipError_t e = ksim_pstream_prepare(&c, h->mirror, ksim_stream(h));
    if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "stream prepare: %s", hipGetErrorString(e));
  }
  const size_t gb = ksim_pfast_granule_bytes();
  if (h->gran_bytes < gb) {
    int rc = dev_alloc(h, &h->granules, gb / sizeof(uint64_t));
    if (rc) return rc;
    h->gran_bytes = gb;
  }
  c.first = first;
  c.end = first + count;
  c.chunk = (c.n + grid - 1) / grid;
  // the cached form (every pod of the range has a tree class, <= 64 classes, the classes'
  // evaluations fit LDS beside the rows, map scores below 2^15): KSIM_NO_PCACHE=1 disables it
  int ncls = 0;
  if (!stream && !getenv("KSIM_NO_PCACHE") && h->n_tcls > 0 && h->tcls && h->tclass) {
    int64_t sw = 0;
    for (int k : {KSIM_W_LEAST_REQUESTED, KSIM_W_MOST_REQUESTED, KSIM_W_BALANCED}) sw += c.no_prio ? 0 : c.w[k] * 10;
    if (sw < 32767 && ksim_pfast_cache_bytes(lds_rows, h->n_tcls)) ncls = h->n_tcls;
  }
  h->last_pfast_cache = ncls > 0;
  HIPCHK(h, hipMemsetAsync(h->granules, 0, gb, ksim_stream(h)));
  HIPCHK(h, hipEventRecord(h->ev0, ksim_stream(h)));
  hipError_t e = ksim_launch_pfast(&c, h->granules, grid, lds_rows, stream ? h->mirror : nullptr, &h->shard, h->tcls,
                                   h->tclass, ncls, ksim_stream(h));
  if (e == hipErrorCooperativeLaunchTooLarge) {
    // the grid cannot be co-resident here (a smaller or shared device): the general kernels instead
    if (h->cfg.mode != KSIM_MODE_PERSISTENT && h->shard.world == 1) {
      h->pfast_off = true;
      return run_persistent_mode(h, first, count, st);
    }
    return ksim_fail(h, KSIM_E_UNSUPPORTED, "persistent launch: %d workgroups cannot be co-resident on this device", grid);
  }
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "persistent launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipEventRecord(h->ev1, ksim_stream(h)));
  HIPCHK(h, hipEventSynchronize(h->ev1));
  float ms = 0.f;
  HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
#ifdef KSIM_STAMPS
  {
    uint64_t d[64];
    HIPCHK(h, hipMemcpy(d, c.dbg, sizeof d, hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemset(c.dbg, 0, sizeof d));
    const double nf = (double)(d[21] ? d[21] : 1);
    {
    fprintf(stderr, "[ksim stamps] pfast workgroup 0, per wave (0 = control) cycles/pod between main barriers busy/wait:");
    for (int w = 0; w < 8; ++w) fprintf(stderr, " %d:%.0f/%.0f", w, d[32 + w] / (double)count, d[40 + w] / (double)count);
    fprintf(stderr, "\n");
    fprintf(stderr, "[ksim stamps] pfast pods=%lld (%.3f ms) cycles/pod: sweep %.0f fix-wait %.0f decide %.0f owner %.0f barrier %.0f "
            "tail %.0f row-eval %.0f; consecutive owners %.3f\n",
            (long long)count, ms, d[2] / (double)count, d[12] / (double)count, d[3] / (double)count, d[6] / (double)count,
            d[7] / (double)count, (d[4] + d[1]) / (double)count, d[5] / (double)count, d[23] / (double)count);
    fprintf(stderr, "[ksim stamps] pfast row wave 1 cycles/pod: pods %.0f eval %.0f wave-stats %.0f publish %.0f\n",
            d[8] / (double)count, d[9] / (double)count, d[10] / (double)count, d[11] / (double)count);
    fprintf(stderr, "[ksim stamps] pfast owner (%llu fixes) cycles: select %.0f barrier %.0f fix-publish %.0f commit+barrier+restat %.0f\n",
            (unsigned long long)d[21], d[22] / nf, d[17] / nf, d[18] / nf, d[19] / nf);
    }
  }
#endif
  if (st) {
    st->device_ms = ms;
    st->kernel_ms = ms;
    st->kernel_launches = 1;
    st->mode = KSIM_MODE_PERSISTENT;
    st->blocks = grid;
  }
  return KSIM_OK;
}

// The general persistent kernel (ksim_pgen.hip) for a range with affinity / spread / volume /
// service-affinity pods: its launch plan, or false when it cannot take the range (the launch form
// then does).  Everything the cycle touches must fit one workgroup's LDS for <= 1,024 rows and
// <= 256 workgroups (co-resident, checked at launch); scores within the granule's 31 bits; the
// spread reduce's zones within one record; every pod-context record within PG_REC_MAX.
struct PgPlan {
  int grid = 0, npt = 0;
  bool v2 = true;  // the dual-hypothesis kernel (192 rows per thread slot); KSIM_PGEN_V1 selects the single one
  int64_t chunk = 0;
  size_t lds = 0;
  PgDims d{};
  uint32_t off[PGO_N] = {};
};

static bool pgen_plan(ksim_handle* h, PgPlan* pl, bool allow_v2 = true) {
  const KsimCtx& c = h->ctx;
  if (getenv("KSIM_NO_PGEN") || h->pgen_off || h->shard.world > 1 || c.n <= 0) return false;
  const bool aux = ksim_rt_aux_on(h), lender = ksim_rt_svc_lender_on(h);
  // the lender check: its totals' domain-0 copies in every workgroup, single-hypothesis kernel only
  if (lender && h->aff_n_pair > PG_SVC_PAIRS) return false;
  if (lender) allow_v2 = false;
  int64_t s = 0;
  for (int k : {KSIM_W_LEAST_REQUESTED, KSIM_W_MOST_REQUESTED, KSIM_W_BALANCED, KSIM_W_INTERPOD_AFFINITY,
                KSIM_W_SELECTOR_SPREAD}) {
    if (c.w[k] > ((int64_t)1 << 30)) return false;
    s += c.w[k] * 10;
  }
  if (aux) {
    if (h->aff_h.aux_w > ((int64_t)1 << 30)) return false;
    s += h->aff_h.aux_w * 10;
  }
  if (s >= ((int64_t)1 << 31)) return false;
  if (h->have_aff) {
    if (c.w[KSIM_W_SELECTOR_SPREAD] && h->aff_n_zone > ksim_pgen_max_zones()) return false;
    // the auxiliary priority: its domain sums in one pass-A record
    if (aux && h->aff_h.n_adom > ksim_pgen_max_aux_domains()) return false;
    if (h->pg_max_mp + h->pg_max_car > 512) return false;  // the shared-domain commit's list
  }
  // the pod-context record bound (ksim_pgen.h): the longest list of every kind
  PgHdr b{};
  if (h->have_aff) {
    b.n_anti = h->pg_max_anti; b.n_prio = h->pg_max_prio; b.n_mp = h->pg_max_mp;
    b.n_req = h->pg_max_req; b.n_pref = h->pg_max_pref; b.n_car = h->pg_max_car;
  }
  if (h->have_vol) {
    b.n_ref = h->vol_max_ref;
    b.n_zw = h->vol_h.zone_ok ? h->vol_h.zone_words : 0;
  }
  b.n_port = h->q_max_port;
  b.n_scal = h->q_max_scal;
  uint32_t so[PGS_END + 1];
  pg_sections(b, so);
  if (so[PGS_END] > PG_REC_MAX) return false;
  PgDims d{};
  d.rec_stride = (int32_t)so[PGS_END];
  d.vcap = h->have_vol ? h->vol_h.vol_slots : 0;
  d.vslots = std::min(d.vcap, PG_VS_LDS);
  d.pslots = c.port_slots;
  if (h->have_aff) { d.n_keys = h->aff_n_keys; d.n_pair = h->aff_n_pair; d.n_carry = h->aff_n_carry; }
  const size_t budget = ksim_pgen_lds_budget();
  const int64_t gcap = (h->max_grid > 0 && h->max_grid < 256) ? h->max_grid : 256;
  int64_t cmin = (c.n + gcap - 1) / gcap;  // at most 256 workgroups (KSIM_MAX_GRID)
  if (cmin > 1024) return false;
  // the dual form: at most 64 workgroups (one granule per lane in its sweeps), 768 rows each
  pl->v2 = allow_v2 && !getenv("KSIM_PGEN_V1") && c.n <= 64 * 768;
  if (pl->v2) cmin = std::max<int64_t>(cmin, (c.n + 63) / 64);
  const int64_t rt = pl->v2 ? 192 : 256;  // rows per thread slot
  d.hyp = pl->v2 ? 1 : 0;
  // the dense hypothesis deltas (E1's count lookups in one step), when small
  const int32_t hdense = (pl->v2 && h->have_aff && !getenv("KSIM_PGEN_NO_HDENSE") &&
                          (int64_t)d.n_pair * 4 + (int64_t)d.n_carry * 12 <= 16384) ? 1 : 0;
  int64_t chunk = std::min<int64_t>(std::max<int64_t>(cmin, rt), c.n);
  if (const char* e = getenv("KSIM_PGEN_CHUNK")) chunk = std::max<int64_t>(cmin, std::min<int64_t>(atoll(e), 4 * rt));
  for (;;) {
    d.n_st = c.n_classes_dev;  // the static (pod class, row) words, when they fit
    d.hdense = hdense;
    size_t lds = ksim_pgen_plan(chunk, &d, pl->off);
    if (lds > budget) {
      d.n_st = 0;
      lds = ksim_pgen_plan(chunk, &d, pl->off);
    }
    if (lds > budget && d.hdense) {
      d.hdense = 0;
      lds = ksim_pgen_plan(chunk, &d, pl->off);
    }
    if (lds <= budget) {
      pl->lds = lds;
      break;
    }
    if (chunk <= cmin) return pl->v2 ? pgen_plan(h, pl, false) : false;
    chunk = std::max<int64_t>(cmin, chunk * 7 / 8);
  }
  pl->chunk = chunk;
  pl->grid = (int)((c.n + chunk - 1) / chunk);
  if (pl->v2 && pl->grid > 64) return pgen_plan(h, pl, false);
  pl->npt = chunk <= rt ? 1 : chunk <= 2 * rt ? 2 : 4;
  pl->d = d;
  return true;
}

// The general persistent kernel over [first, first+count): the pod-context records are packed,
// then one launch schedules the range; the kernel writes the node rows, volume slots, host ports
// and canonical affinity counts back to HBM at its end.
static int run_pgen_mode(ksim_handle* h, int64_t first, int64_t count, const PgPlan& pl, ksim_stats* st) {
  KsimCtx& c = h->ctx;
  int rc;
  const size_t gb = ksim_pgen_gran_bytes();
  if (!h->pg_gran && (rc = dev_alloc(h, &h->pg_gran, gb / sizeof(uint64_t)))) return rc;
  const size_t rb = (size_t)count * pl.d.rec_stride;
  if (h->pg_rec_bytes < rb) {
    if (h->pg_rec) dev_free(h, h->pg_rec);
    h->pg_rec = nullptr;
    h->pg_rec_bytes = 0;
    if ((rc = dev_alloc(h, &h->pg_rec, std::max<size_t>(rb, 1 << 20)))) return rc;
    h->pg_rec_bytes = std::max<size_t>(rb, 1 << 20);
  }
  PGenArgs g{};
  g.gran = h->pg_gran;
  g.rec = h->pg_rec;
  g.spin_ticks = 200000000ull;  // 2 s per wait
  if (const char* e = getenv("KSIM_PGEN_SPIN_TICKS")) g.spin_ticks = strtoull(e, nullptr, 10);
  g.test_stall = getenv("KSIM_PGEN_TEST_STALL") ? 1 : 0;
  g.d = pl.d;
  memcpy(g.off, pl.off, sizeof g.off);
  g.has_vol = h->have_vol ? 1 : 0;
  if (h->have_vol) g.V = h->vol_h;
  g.svc_on = ksim_rt_svc_lender_on(h) ? 1 : 0;
  if (h->have_aff) {
    g.ident_shared = h->aff_ident_shared;
    g.aclass_shared = h->aff_aclass_shared;
    g.id_anti_off = h->pg_id_anti_off; g.id_anti = h->pg_id_anti;
    g.id_prio_off = h->pg_id_prio_off; g.id_prio = h->pg_id_prio;
    g.id_mp_off = h->pg_id_mp_off; g.id_mp = h->pg_id_mp;
    g.n_zone = h->aff_n_zone;
    g.has_aff = 1;
    g.A = h->aff_h;
  }
  c.first = first;
  c.end = first + count;
  c.chunk = pl.chunk;
  HIPCHK(h, hipMemsetAsync(h->pg_gran, 0, gb, ksim_stream(h)));
  const int64_t end = first + count;  // the kernel lowers the cursor to the first pod it did not schedule
  HIPCHK(h, hipMemcpyAsync(c.cursor, &end, 8, hipMemcpyHostToDevice, ksim_stream(h)));
  HIPCHK(h, hipEventRecord(h->ev0, ksim_stream(h)));
  hipError_t e = ksim_pgen_pack(&c, &g, ksim_stream(h));
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "pgen pack: %s", hipGetErrorString(e));
  e = pl.v2 ? ksim_launch_pgen2(&c, &g, pl.grid, pl.npt, pl.lds, ksim_stream(h))
            : ksim_launch_pgen(&c, &g, pl.grid, pl.npt, pl.lds, ksim_stream(h));
  if (e == hipErrorCooperativeLaunchTooLarge) {
    if (h->cfg.mode != KSIM_MODE_PERSISTENT) return run_launch_mode(h, first, count, st);
    return ksim_fail(h, KSIM_E_UNSUPPORTED, "persistent launch: %d workgroups cannot be co-resident on this device", pl.grid);
  }
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "pgen launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipEventRecord(h->ev1, ksim_stream(h)));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  float ms = 0.f;
  HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
#ifdef KSIM_STAMPS
  {
    uint64_t dd[64];
    HIPCHK(h, hipMemcpy(dd, c.dbg, sizeof dd, hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemset(c.dbg, 0, sizeof dd));
    fprintf(stderr, "[ksim stamps] pgen pods=%lld (%.3f ms, grid %d, chunk %lld, st %d, hdense %d, rec %d B, lds %zu) cycles/pod: eval %.0f "
            "passA-local %.0f passA-xchg %.0f classes %.0f class-sweep %.0f decide %.0f pick+commit %.0f aff-shared %.0f\n",
            (long long)count, ms, pl.grid, (long long)pl.chunk, pl.d.n_st, pl.d.hdense, pl.d.rec_stride, pl.lds, dd[0] / (double)count,
            dd[6] / (double)count, dd[1] / (double)count, dd[2] / (double)count, dd[7] / (double)count, dd[3] / (double)count,
            dd[4] / (double)count, dd[5] / (double)count);
    fprintf(stderr, "[ksim stamps] pgen eval split (thread 0's row) cycles/pod: top+row %.0f predicates %.0f map %.0f\n",
            dd[8] / (double)count, dd[9] / (double)count, dd[10] / (double)count);
    fprintf(stderr, "[ksim stamps] pgen decide split (wave 0 of workgroup 0) cycles/pod: per-class %.0f rest %.0f barrier %.0f\n",
            dd[11] / (double)count, dd[12] / (double)count, dd[3] / (double)count);
    if (pl.v2)
      fprintf(stderr, "[ksim stamps] pgen2 over workgroups cycles/pod max/min: passA-xchg %.0f/%.0f classes %.0f/%.0f decide-window "
              "%.0f/%.0f passA-local %.0f/%.0f row-eval %.0f/%.0f\n",
              dd[16] / (double)count, ~dd[17] / (double)count, dd[18] / (double)count, ~dd[19] / (double)count,
              dd[20] / (double)count, ~dd[21] / (double)count, dd[22] / (double)count, ~dd[23] / (double)count,
              dd[24] / (double)count, ~dd[25] / (double)count);
    if (pl.v2)
      fprintf(stderr, "[ksim stamps] pgen2 mean over workgroups cycles/pod: passA spin %.0f passA reduce %.0f class spin %.0f; "
              "deferred commit %.0f cycles each (%.0f commits)\n",
              dd[33] / (double)count / pl.grid, dd[34] / (double)count / pl.grid, dd[35] / (double)count / pl.grid,
              dd[36] ? dd[32] / (double)dd[36] : 0.0, (double)dd[36]);
    if (pl.v2)
      fprintf(stderr, "[ksim stamps] pgen2 E1 waves (thread 320) cycles/pod max/min: %.0f/%.0f\n", dd[14] / (double)count,
              ~dd[15] / (double)count);
    if (pl.v2)
      fprintf(stderr, "[ksim stamps] pgen2 row eval split (threads 64 + 320, mean over workgroups, E0+E1) cycles/pod: row+static %.0f "
              "ports+resources %.0f disk-conflict %.0f taints..max-volumes %.0f pressure+interpod %.0f map+ipa+spread %.0f\n",
              dd[26] / (double)count / pl.grid, dd[27] / (double)count / pl.grid, dd[28] / (double)count / pl.grid,
              dd[29] / (double)count / pl.grid, dd[30] / (double)count / pl.grid, dd[31] / (double)count / pl.grid);
  }
#endif
  if (st) {
    st->device_ms = ms;
    st->kernel_ms = ms;
    st->kernel_launches = 1;
    st->mode = KSIM_MODE_PERSISTENT;
    st->blocks = pl.grid;
  }
  int32_t err = 0;
  HIPCHK(h, hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
  if (err & 4) {
    // a spin bound ran out (the grid was not co-resident after all, e.g. another process's kernels
    // held CUs): every workgroup stopped before deciding the pod at the cursor and wrote back what
    // it had committed.  Clear the bit and finish [cursor, end) with the launch form; the general
    // persistent kernel stays off for this handle.
    int64_t cur = end;
    HIPCHK(h, hipMemcpy(&cur, c.cursor, 8, hipMemcpyDeviceToHost));
    err &= ~4;
    HIPCHK(h, hipMemcpy(c.err, &err, 4, hipMemcpyHostToDevice));
    h->pgen_off = true;
    if (cur < first || cur > end) return ksim_fail(h, KSIM_E_DEVICE, "pgen abort at an impossible pod %lld", (long long)cur);
    if (cur < end) {
      ksim_stats s2{};
      if ((rc = run_launch_mode(h, cur, end - cur, &s2))) return rc;
      if (st) {
        st->device_ms += s2.device_ms;
        st->kernel_ms += s2.kernel_ms;
        st->kernel_launches += s2.kernel_launches;
        st->mode = KSIM_MODE_LAUNCH;
      }
    }
  }
  return KSIM_OK;
}

// Pods only the launch kernels or the general persistent kernel schedule (affinity, volumes,
// service affinity): the persistent one when it can take the range.
static int run_f3_range(ksim_handle* h, int64_t first, int64_t count, ksim_stats* st) {
  PgPlan pl;
  if (h->cfg.mode == KSIM_MODE_LAUNCH || !pgen_plan(h, &pl)) return run_launch_mode(h, first, count, st);
  // the pod-context records (up to PG_REC_MAX bytes per pod) of at most ~256 MB per launch: a long
  // range goes in sub-ranges (the table, slots and counts persist in HBM between launches)
  const int64_t per = std::max<int64_t>(1, ((int64_t)256 << 20) / std::max<int64_t>(pl.d.rec_stride, 1));
  if (st) memset(st, 0, sizeof *st);
  for (int64_t a = first; a < first + count; a += per) {
    const int64_t n = std::min<int64_t>(per, first + count - a);
    ksim_stats s2{};
    int rc = h->pgen_off ? run_launch_mode(h, a, n, &s2) : run_pgen_mode(h, a, n, pl, &s2);
    if (rc) return rc;
    if (st) {
      st->device_ms += s2.device_ms;
      st->kernel_ms += s2.kernel_ms;
      st->kernel_launches += s2.kernel_launches;
      st->mode = s2.mode;
      st->blocks = s2.blocks;
    }
  }
  return KSIM_OK;
}

static int run_persistent_mode(ksim_handle* h, int64_t first, int64_t count, ksim_stats* st) {
  KsimCtx& c = h->ctx;
  // inter-pod affinity, volume and service-affinity pods, and every pod under the auxiliary
  // priority: the general persistent kernel (or the launch form)
  if (ksim_rt_aux_on(h) || ksim_rt_launch_only_count(h, first, count)) return run_f3_range(h, first, count, st);
  int grid = 0, lds_rows = 0;
  if (const int form = pfast_form(h, first, count, &grid, &lds_rows)) {
    int rc = run_pfast_mode(h, first, count, grid, lds_rows, form == 2, st);
    if (rc) return rc;
    int32_t err = 0;
    HIPCHK(h, hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
    if (!(err & 8)) return KSIM_OK;
    // a node left the exact float64 range: the general kernel from now on
    h->pfast_off = true;
    int64_t cur = 0;
    HIPCHK(h, hipMemcpy(&cur, c.cursor, 8, hipMemcpyDeviceToHost));
    err &= ~8;
    HIPCHK(h, hipMemcpy(c.err, &err, 4, hipMemcpyHostToDevice));
    if (cur >= first + count) return KSIM_OK;
    const double ms0 = st ? st->kernel_ms : 0.0;
    ksim_stats s2{};
    rc = run_persistent_mode(h, cur, first + count - cur, &s2);
    if (rc) return rc;
    if (st) {
      st->device_ms += s2.device_ms;
      st->kernel_ms = ms0 + s2.kernel_ms;
      st->kernel_launches += s2.kernel_launches;
    }
    return KSIM_OK;
  }
  if (!ksim_persistent_config(c.n, &grid, &lds_rows)) {
    // the streaming fast kernel handed over (a node left the exact float64 range): the
    // general kernel of a table this size is the launch form
    if (h->pfast_off && h->cfg.mode != KSIM_MODE_PERSISTENT) return run_launch_mode(h, first, count, st);
    return ksim_fail(h, KSIM_E_UNSUPPORTED, "persistent mode: node table does not fit the on-chip layout");
  }
  if (!persistent_weights_ok(c)) return ksim_fail(h, KSIM_E_UNSUPPORTED, "persistent mode: map-priority weights exceed the 27-bit score range");
  const size_t gb = ksim_persistent_granule_bytes(grid);
  if (h->gran_bytes < gb) {
    int rc = dev_alloc(h, &h->granules, gb / sizeof(uint64_t));
    if (rc) return rc;
    h->gran_bytes = gb;
  }
  c.first = first;
  c.end = first + count;
  c.chunk = (c.n + grid - 1) / grid;
  if (!h->ctx_dev) {
    int rc = dev_alloc(h, &h->ctx_dev, 1);
    if (rc) return rc;
  }
  HIPCHK(h, hipMemcpyAsync(h->ctx_dev, &c, sizeof(KsimCtx), hipMemcpyHostToDevice, ksim_stream(h)));
  HIPCHK(h, hipMemsetAsync(h->granules, 0, gb, ksim_stream(h)));
  HIPCHK(h, hipEventRecord(h->ev0, ksim_stream(h)));
  hipError_t e = ksim_launch_persistent(&c, h->ctx_dev, h->granules, grid, lds_rows, ksim_stream(h));
  if (e == hipErrorCooperativeLaunchTooLarge) {
    // the grid cannot be co-resident here (a smaller or shared device): the launch form instead
    if (h->cfg.mode != KSIM_MODE_PERSISTENT && h->shard.world == 1) return run_launch_mode(h, first, count, st);
    return ksim_fail(h, KSIM_E_UNSUPPORTED, "persistent launch: %d workgroups cannot be co-resident on this device", grid);
  }
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "persistent launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipEventRecord(h->ev1, ksim_stream(h)));
  HIPCHK(h, hipEventSynchronize(h->ev1));
  float ms = 0.f;
  HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
#ifdef KSIM_STAMPS
  {
    uint64_t d[32];
    HIPCHK(h, hipMemcpy(d, c.dbg, sizeof d, hipMemcpyDeviceToHost));
    HIPCHK(h, hipMemset(c.dbg, 0, sizeof d));
    // slots: 1 publish, 2 sweep, 9 reduce, 10 selectHost index, 3 locate, 6 select+commit,
    // 7 barrier, 11 fix-up, 4 combine, 5 row-wave evaluation (concurrent), 8 polls
    static const char* names[16] = {"", "publish", "sweep", "locate", "combine", "row-eval", "select+commit", "barrier",
                                    "polls", "reduce", "ix", "classes", "spec-seen", "fix-seen", "", ""};
    fprintf(stderr, "[ksim stamps] pods=%lld (%.3f ms) cycles/pod:", (long long)count, ms);
    for (int k : {1, 2, 12, 13, 9, 11, 10, 3, 6, 7, 4, 5, 8}) fprintf(stderr, " %s %.0f", names[k], d[k] / (double)count);
    fprintf(stderr, "\n[ksim stamps] row wave 1: eval %.0f partial %.0f", d[24] / (double)count, d[25] / (double)count);
    fprintf(stderr, " (per call: view %.0f rows %.0f read-back %.0f)", d[26] / (double)(d[29] ? d[29] : 1),
            d[27] / (double)(d[29] ? d[29] : 1), d[28] / (double)(d[29] ? d[29] : 1));
    fprintf(stderr, " wait for control %.0f", d[30] / (double)count);
    fprintf(stderr, "\n[ksim stamps] owner select %.0f commit %.0f", d[22] / (double)(d[21] ? d[21] : 1),
            d[23] / (double)(d[21] ? d[21] : 1));
    fprintf(stderr, "\n[ksim stamps] owner (%llu fix-ups) cycles/fix-up: pre-eval %.0f barrier %.0f eval-row %.0f partial %.0f combine+publish %.0f\n",
            (unsigned long long)d[21], d[16] / (double)(d[21] ? d[21] : 1), d[17] / (double)(d[21] ? d[21] : 1),
            d[18] / (double)(d[21] ? d[21] : 1), d[19] / (double)(d[21] ? d[21] : 1), d[20] / (double)(d[21] ? d[21] : 1));
  }
#endif
  if (st) {
    st->device_ms = ms;
    st->kernel_ms = ms;
    st->kernel_launches = 1;
    st->mode = KSIM_MODE_PERSISTENT;
    st->blocks = grid;
  }
  return KSIM_OK;
}

// AUTO dispatch: the persistent kernels when the table fits on chip (or the streaming fast
// kernel can take the range), else the launch form.
static int run_auto_mode(ksim_handle* h, int64_t first, int64_t count, ksim_stats* st) {
  int g, l;
  // (the auxiliary priority: every pod to the general kernels — a serviceAntiAffinity priority
  // scores pods no service selects too)
  if (ksim_rt_aux_on(h) || ksim_rt_launch_only_count(h, first, count)) {
    h->tree_valid = false;
    return run_f3_range(h, first, count, st);
  }
  const bool pers = (ksim_persistent_config(h->ctx.n, &g, &l) && persistent_weights_ok(h->ctx)) ||
                    pfast_form(h, first, count, &g, &l);
  h->tree_valid = false;  // these paths commit without maintaining the trees
  return pers ? run_persistent_mode(h, first, count, st) : run_launch_mode(h, first, count, st);
}

// Can tree mode run at all on this handle (one device, class set and weights within the tree's
// packing, every quantity exact in float64)?  Plans the geometry and allocates the trees once.
static int tree_ready(ksim_handle* h, bool* ok) {
  *ok = false;
  const KsimCtx& c = h->ctx;
  if (h->shard.world > 1 || h->n_tcls <= 0 || h->pfast_off || getenv("KSIM_NO_TREE")) return KSIM_OK;
  if (!c.no_prio) {
    int64_t s = 0;
    for (int k : {KSIM_W_LEAST_REQUESTED, KSIM_W_MOST_REQUESTED, KSIM_W_BALANCED}) {
      if (c.w[k] > 65535) return KSIM_OK;
      s += c.w[k] * 10;
    }
    if (s > 65534) return KSIM_OK;  // (score + 1) packs into 16 bits
  }
  if (!h->tree_planned) {
    h->tree_planned = true;
    const char* lb = getenv("KSIM_TREE_LDS");  // tests: force global levels on small tables
    const char* fm = getenv("KSIM_TREE_M");
    h->tree_ok = ksim_tree_plan(c.n, h->n_tcls, lb ? atoll(lb) : 0, fm ? atoi(fm) : 0, &h->geo) != 0;
    if (h->tree_ok) {
      int rc;
      if ((rc = dev_alloc(h, &h->t_leaves, (size_t)h->geo.K * h->geo.st[0])) ||
          (rc = dev_alloc(h, &h->t_levels, (size_t)h->geo.level_entries)) ||
          (rc = dev_alloc(h, &h->t_fit, (size_t)h->geo.K)) || (rc = dev_alloc(h, &h->t_y, (size_t)2 * c.n)))
        return rc;
    }
  }
  *ok = h->tree_ok;
  return KSIM_OK;
}

static void add_stats(ksim_stats* st, const ksim_stats& s) {
  if (!st) return;
  st->device_ms += s.device_ms;
  st->kernel_ms += s.kernel_ms;
  st->kernel_launches += s.kernel_launches;
  if (!st->mode) { st->mode = s.mode; st->blocks = s.blocks; }
}

// Tree mode (ksim_tree.hip): maximal runs of resource-only pods go to the tree kernel (trees
// rebuilt first if another path committed since), other runs to the AUTO path.
static int run_tree_mode(ksim_handle* h, int64_t first, int64_t count, ksim_stats* st) {
  KsimCtx& c = h->ctx;
  bool ok = false;
  int rc = tree_ready(h, &ok);
  if (rc) return rc;
  if (!ok) return run_auto_mode(h, first, count, st);
  if (st) memset(st, 0, sizeof *st);
  const int64_t end = first + count;
  auto fast = [&](int64_t i) { return h->fast_pre[i + 1] != h->fast_pre[i]; };
  int64_t i = first;
  while (i < end) {
    int64_t j = i;
    while (j < end && fast(j)) ++j;
    if (j == i || h->pfast_off) {  // a run of other pods (or the tree stopped for good)
      if (j == i)
        while (j < end && !fast(j)) ++j;
      ksim_stats s2{};
      if ((rc = run_auto_mode(h, i, j - i, &s2))) return rc;
      add_stats(st, s2);
      // a failure of that segment (overflow, inconsistency) ends the call here: ksim_schedule reports
      // it before any later segment could read or clear the error word
      int32_t err = 0;
      HIPCHK(h, hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
      if (err) return KSIM_OK;
      i = j;
      continue;
    }
    HIPCHK(h, hipEventRecord(h->ev0, ksim_stream(h)));
    if (!h->tree_valid) {
      hipError_t e = ksim_tree_build(&c, &h->geo, h->tclass, h->tcls, h->t_leaves, h->t_levels, h->t_fit, h->t_y, nullptr, ksim_stream(h));
      if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "tree build: %s", hipGetErrorString(e));
    }
    c.first = i;
    c.end = j;
    HIPCHK(h, hipEventRecord(h->ev1, ksim_stream(h)));
    hipError_t e = ksim_tree_launch(&c, &h->geo, h->tclass, h->tcls, h->t_leaves, h->t_levels, h->t_fit, h->t_y, nullptr, ksim_stream(h));
    if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "tree launch: %s", hipGetErrorString(e));
    hipEvent_t ev2 = nullptr;
    HIPCHK(h, hipEventCreate(&ev2));
    HIPCHK(h, hipEventRecord(ev2, ksim_stream(h)));
    HIPCHK(h, hipEventSynchronize(ev2));
    float build_ms = 0.f, run_ms = 0.f;
    HIPCHK(h, hipEventElapsedTime(&build_ms, h->ev0, h->ev1));
    HIPCHK(h, hipEventElapsedTime(&run_ms, h->ev1, ev2));
    (void)hipEventDestroy(ev2);
    if (st) {
      st->device_ms += build_ms + run_ms;
      st->kernel_ms += run_ms;
      st->kernel_launches += 1;
      st->mode = KSIM_MODE_TREE;
      st->blocks = 1;
    }
#ifdef KSIM_STAMPS
    {
      uint64_t d[32];
      HIPCHK(h, hipMemcpy(d, c.dbg, sizeof d, hipMemcpyDeviceToHost));
      HIPCHK(h, hipMemset(c.dbg, 0, sizeof d));
      const double np = (double)(d[8] ? d[8] : 1);
      fprintf(stderr, "[ksim stamps] tree pods=%llu (%.3f ms) cycles/pod: decide %.0f walk (levels %.0f, leaf load %.0f, leaf "
              "pick %.0f) row+eval %.0f paths %.0f; changed classes %.2f, re-combined paths %.3f per pod\n",
              (unsigned long long)d[8], run_ms, d[0] / np, d[4] / np, d[5] / np, d[1] / np, d[2] / np, d[3] / np,
              d[6] / np, d[7] / np);
    }
#endif
    int32_t err = 0;
    HIPCHK(h, hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
    if (err & 16) return ksim_fail(h, KSIM_E_DEVICE, "tree mode: tree inconsistent with its root (0x%x)", err);
    h->tree_valid = true;
    if (err & 8) {  // a node's quantities left the exact float64 range: the general kernels from now on
      h->pfast_off = true;
      h->tree_valid = false;
      err &= ~8;
      HIPCHK(h, hipMemcpy(c.err, &err, 4, hipMemcpyHostToDevice));
      int64_t cur = 0;
      HIPCHK(h, hipMemcpy(&cur, c.cursor, 8, hipMemcpyDeviceToHost));
      j = cur;
    }
    i = j;
  }
  return KSIM_OK;
}

extern "C" {

int ksim_schedule(ksim_handle* h, int64_t first, int64_t count, int32_t* out_node, int32_t* out_reasons,
                  ksim_stats* st) {
  if (!h) return ksim_fail(h, KSIM_E_INVAL, "ksim_schedule: null handle");
  if (!h->have_pods) return ksim_fail(h, KSIM_E_STATE, "ksim_schedule: load nodes, classes and pods first");
  if (first < 0 || count < 0 || first + count > h->n_pods) return ksim_fail(h, KSIM_E_INVAL, "ksim_schedule: range out of bounds");
  HIPCHK(h, hipSetDevice(h->device));
  if (st) memset(st, 0, sizeof *st);
  if (count == 0) return KSIM_OK;
  KsimCtx& c = h->ctx;
  if (c.n == 0) return ksim_fail(h, KSIM_E_NO_NODES, "no nodes available to schedule pods");
  if (int rc = ksim_rt_check_aff(h, "ksim_schedule")) return rc;
  KsimGate gate(h, true);  // the persistent kernels' workgroups wait on each other
  if (h->shard.world > 1) {  // node-sharded: the fast persistent kernel on every rank, in lockstep
    for (int r = 0; r < h->shard.world; ++r)
      if (!h->shard.peers[r]) return ksim_fail(h, KSIM_E_STATE, "ksim_schedule: rank %d is not connected", r);
    int grid = 0, lds_rows = 0;
    // (the auxiliary priority: every pod to the launch form — a serviceAntiAffinity priority scores
    // pods no service selects too)
    const int form = ksim_rt_aux_on(h) ? 0 : pfast_form(h, first, count, &grid, &lds_rows);
    int rc;
    if (form) {
      rc = run_pfast_mode(h, first, count, grid, lds_rows, form == 2, st);
    } else {
      // pods beyond the fast kernel (selectors, taints, ports, reduce classes): the launch form,
      // exchanging each pod's decision inputs across the ranks (SURVEY.md §8e Phase A)
      if (ksim_rt_range_wide(h, first, count))
        return ksim_fail(h, KSIM_E_UNSUPPORTED, "node-sharded scheduling of pods with more than %d reduce classes",
                         KSIM_MAX_RCLASS);
      if (ksim_rt_svc_lender_on(h) || (h->have_aff && h->aff_h.n_zone > KSIM_PX_ZONES) ||
          (ksim_rt_aux_on(h) && h->aff_h.n_adom > KSIM_PX_ADOMS))
        return ksim_fail(h, KSIM_E_UNSUPPORTED, "node-sharded scheduling with the service-affinity lender check, more than "
                                           "%d spread zones or more than %d auxiliary-priority domains", KSIM_PX_ZONES,
                         KSIM_PX_ADOMS);
      // per-node scores travel as 40-bit biased words (KSIM_LX_BIAS = 2^39): every weight that
      // reaches a node's score is bounded, and so is their sum x MaxPriority
      {
        int64_t sw = 0;
        for (int k : {KSIM_W_LEAST_REQUESTED, KSIM_W_MOST_REQUESTED, KSIM_W_BALANCED, KSIM_W_INTERPOD_AFFINITY,
                      KSIM_W_SELECTOR_SPREAD}) {
          if (c.w[k] > ((int64_t)1 << 30))
            return ksim_fail(h, KSIM_E_UNSUPPORTED, "node-sharded scheduling: a priority weight above 2^30");
          sw += c.w[k] * 10;
        }
        if (ksim_rt_aux_on(h)) {
          if (h->aff_h.aux_w > ((int64_t)1 << 30))
            return ksim_fail(h, KSIM_E_UNSUPPORTED, "node-sharded scheduling: a priority weight above 2^30");
          sw += h->aff_h.aux_w * 10;
        }
        if (sw >= ((int64_t)1 << 39))
          return ksim_fail(h, KSIM_E_UNSUPPORTED, "node-sharded scheduling: weighted scores beyond the 40-bit exchange word");
      }
      c.sh_world = h->shard.world;
      c.sh_rank = h->shard.rank;
      c.sh_base = h->shard.node_base;
      c.sh_tag0 = h->shard.xtag_base;
      c.sh_start_ticks = h->shard.start_ticks;
      for (int r = 0; r < KSIM_MAX_RANKS; ++r)
        c.sh_peers[r] = h->shard.peers[r] ? h->shard.peers[r] + ksim_shard_lx_offset() : nullptr;
      // the tags are baked into the launch graph's arguments: capture it again for this call
      if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
      if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
      rc = run_launch_mode(h, first, count, st);
      c.sh_world = 0;
      if (h->gexec) { (void)hipGraphExecDestroy(h->gexec); h->gexec = nullptr; }
      if (h->graph) { (void)hipGraphDestroy(h->graph); h->graph = nullptr; }
    }
    h->shard.xtag_base += (uint32_t)count;
    if (rc) return rc;
    int32_t err = 0;
    HIPCHK(h, hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
    if (err & 8) {
      h->pfast_off = true;
      return ksim_fail(h, KSIM_E_UNSUPPORTED, "node-sharded run stopped: a node's quantities left the exact float64 range");
    }
  } else {
  // the auxiliary priority and the service-affinity lender check (ksim_affinity_tables.aux_* /
  // svc_*) are read by the launch-form kernels and the general persistent kernel (tree mode, for
  // pods without them, gives way to the automatic choice)
  const int mode = ksim_rt_range_wide(h, first, count)                          ? KSIM_MODE_LAUNCH
                   : (ksim_rt_launch_tables(h) && h->cfg.mode == KSIM_MODE_TREE) ? KSIM_MODE_AUTO
                                                                                 : h->cfg.mode;
  int rc = mode == KSIM_MODE_TREE         ? run_tree_mode(h, first, count, st)
           : mode == KSIM_MODE_AUTO       ? run_auto_mode(h, first, count, st)
           : mode == KSIM_MODE_PERSISTENT ? run_persistent_mode(h, first, count, st)
                                          : run_launch_mode(h, first, count, st);
  if (mode != KSIM_MODE_TREE) h->tree_valid = false;
  if (rc) return rc;
  }
  int32_t err = 0;
  HIPCHK(h, hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
  if (out_node) HIPCHK(h, hipMemcpy(out_node, c.out_node + first, count * sizeof(int32_t), hipMemcpyDeviceToHost));
  if (out_reasons && c.collect)
    HIPCHK(h, hipMemcpy(out_reasons, c.out_reasons + first * KSIM_NREASONS, count * KSIM_NREASONS * sizeof(int32_t),
                        hipMemcpyDeviceToHost));
  if (st) {
    st->pods = count;
    st->node_evals = count * c.n;
    if (out_node) {
      int64_t s = 0;
      for (int64_t i = 0; i < count; ++i) s += out_node[i] >= 0;
      st->scheduled = s;
    }
  }
  if (err & 1) return ksim_fail(h, KSIM_E_OVERFLOW, "a node's host-port or volume slots overflowed (raise port_slots / vol_slots)");
  if (err & 128) return ksim_rt_svc_refusal(h);
  if (err & ~1) {
    return ksim_fail(h, KSIM_E_DEVICE, "device consistency error 0x%x", err);
  }
  return KSIM_OK;
}

int ksim_evaluate(ksim_handle* h, int64_t pod, uint8_t* out_fit, uint32_t* out_reasons, int64_t* out_score,
                  uint8_t* out_rclass) {
  if (!h) return ksim_fail(h, KSIM_E_INVAL, "ksim_evaluate: null handle");
  if (!h->have_pods) return ksim_fail(h, KSIM_E_STATE, "ksim_evaluate: nothing loaded");
  if (pod < 0 || pod >= h->n_pods) return ksim_fail(h, KSIM_E_INVAL, "ksim_evaluate: pod out of range");
  HIPCHK(h, hipSetDevice(h->device));
  KsimCtx& c = h->ctx;
  const int64_t n = c.n;
  if (n == 0) return ksim_fail(h, KSIM_E_NO_NODES, "no nodes available to schedule pods");
  if (int rc0 = ksim_rt_check_aff(h, "ksim_evaluate")) return rc0;
  uint8_t *f, *rcl;
  uint32_t* r;
  int64_t* s;
  // scratch buffers (kept for the handle's lifetime; small compared with the table)
  int rc;
  if ((rc = dev_alloc(h, &f, n)) || (rc = dev_alloc(h, &r, n)) || (rc = dev_alloc(h, &s, n)) || (rc = dev_alloc(h, &rcl, n)))
    return rc;
  hipError_t e = ksim_launch_eval(&c, pod, f, r, s, rcl, ksim_stream(h));
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "eval launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  if (out_fit) HIPCHK(h, hipMemcpy(out_fit, f, n, hipMemcpyDeviceToHost));
  if (out_reasons) HIPCHK(h, hipMemcpy(out_reasons, r, n * 4, hipMemcpyDeviceToHost));
  if (out_score) HIPCHK(h, hipMemcpy(out_score, s, n * 8, hipMemcpyDeviceToHost));
  if (out_rclass) HIPCHK(h, hipMemcpy(out_rclass, rcl, n, hipMemcpyDeviceToHost));
  // release the scratch buffers again
  for (void* p : {(void*)f, (void*)r, (void*)s, (void*)rcl}) dev_free(h, p);
  return KSIM_OK;
}

int ksim_sweep(ksim_handle* h, const int64_t* weights, int32_t n_scen, int64_t first, int64_t count, int32_t* out_node,
               uint64_t* out_counters, ksim_stats* st) {
  if (!h || !weights || !out_node) return ksim_fail(h, KSIM_E_INVAL, "ksim_sweep: null argument");
  if (!h->have_pods) return ksim_fail(h, KSIM_E_STATE, "ksim_sweep: load nodes, classes and pods first");
  if (n_scen <= 0 || first < 0 || count <= 0 || first + count > h->n_pods || count > INT32_MAX)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_sweep: bad scenario count or pod range");
  HIPCHK(h, hipSetDevice(h->device));
  KsimCtx& c = h->ctx;
  const int64_t n = c.n;
  if (n == 0) return ksim_fail(h, KSIM_E_NO_NODES, "no nodes available to schedule pods");
  if (int rc0 = ksim_rt_check_aff(h, "ksim_sweep")) return rc0;
  if (n > KSIM_SWEEP_MAX_NODES)
    return ksim_fail(h, KSIM_E_UNSUPPORTED, "ksim_sweep: %lld nodes exceed the %d-node scenario layout", (long long)n,
                KSIM_SWEEP_MAX_NODES);
  if (h->fast_pre[first + count] - h->fast_pre[first] != count)
    return ksim_fail(h, KSIM_E_UNSUPPORTED, "ksim_sweep: every pod must be resource-only (no ports, selectors, taints, "
                                       "nodeName, gpu / ephemeral / extended requests)");
  std::vector<int32_t> w3((size_t)n_scen * 3);
  for (int32_t sidx = 0; sidx < n_scen; ++sidx) {
    const int64_t* w = weights + (size_t)sidx * KSIM_NW;
    if (w[KSIM_W_TAINT_TOLERATION] || w[KSIM_W_NODE_AFFINITY])
      return ksim_fail(h, KSIM_E_UNSUPPORTED, "ksim_sweep: scenario %d: reduce priorities are not swept", sidx);
    int64_t tot = 0;
    for (int k : {KSIM_W_LEAST_REQUESTED, KSIM_W_MOST_REQUESTED, KSIM_W_BALANCED}) {
      if (w[k] < 0 || w[k] > 6553) return ksim_fail(h, KSIM_E_UNSUPPORTED, "ksim_sweep: scenario %d: weight out of range", sidx);
      tot += w[k];
    }
    if (tot * 10 >= 0xFFFF) return ksim_fail(h, KSIM_E_UNSUPPORTED, "ksim_sweep: scenario %d: scores exceed 16 bits", sidx);
    w3[3 * sidx] = (int32_t)w[KSIM_W_LEAST_REQUESTED];
    w3[3 * sidx + 1] = (int32_t)w[KSIM_W_MOST_REQUESTED];
    w3[3 * sidx + 2] = (int32_t)w[KSIM_W_BALANCED];
  }
  // float64 exactness: node quantities + count x the largest pod quantity stay below 2^48
  {
    int64_t qmax = 0, nmax = 0;
    for (int64_t i = first; i < first + count; ++i) qmax = std::max(qmax, h->pod_qmax[i]);
    std::vector<int64_t> col((size_t)n);
    for (const int64_t* d : {c.alloc_cpu, c.alloc_mem, (const int64_t*)c.req_cpu, (const int64_t*)c.req_mem,
                             (const int64_t*)c.nz_cpu, (const int64_t*)c.nz_mem}) {
      HIPCHK(h, hipMemcpy(col.data(), d, (size_t)n * 8, hipMemcpyDeviceToHost));
      for (int64_t v : col) nmax = std::max(nmax, v < 0 ? INT64_MAX / 2 : v);
    }
    const int64_t lim = (int64_t)1 << 48;
    if (nmax >= lim || qmax >= lim || count > lim / std::max<int64_t>(qmax, 1) || nmax + count * qmax >= lim)
      return ksim_fail(h, KSIM_E_UNSUPPORTED, "ksim_sweep: quantities may leave the exact float64 range (2^48)");
  }
  int rc;
  // Tree form (ksim_tree.hip): one tree-mode wave per scenario, scenarios spread over the CUs.
  if (!getenv("KSIM_SWEEP_SCAN") && h->n_tcls > 0 && n < ((int64_t)1 << 24) && !h->pfast_off) {
    KsimTreeGeo g{};
    // a small LDS plan: several scenarios' waves per CU hide each other's memory latency
    const char* lb = getenv("KSIM_SWEEP_LDS");
    if (ksim_tree_plan(n, h->n_tcls, lb ? atoll(lb) : 24 * 1024, 0, &g) || ksim_tree_plan(n, h->n_tcls, 0, 0, &g)) {
      if (!h->t_y && (rc = dev_alloc(h, &h->t_y, (size_t)2 * n))) return rc;
      auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
      const size_t N = (size_t)n, P = (size_t)count, K = (size_t)g.K;
      const size_t per = al(4 * N * 8) + al(N * 4) + al(K * g.st[0] * 4) + al(g.level_entries * 8) + al(K * 4) + al(8) +
                         al(P * 4) + al(sizeof(kf64::EvCfg));
      // scratch budget: at most 24 GiB (all 4,096 C5 scenarios, ~3.7 MB each, in one launch) and
      // at most half of the device memory free now (a shared or smaller device gets smaller chunks)
      size_t budget = (size_t)24 << 30, mfree = 0, mtotal = 0;
      if (hipMemGetInfo(&mfree, &mtotal) == hipSuccess && mfree / 2 < budget) budget = mfree / 2;
      int32_t chunk = (int32_t)std::max<size_t>(1, std::min<size_t>((size_t)n_scen, budget / per));
      if (const char* ch = getenv("KSIM_SWEEP_CHUNK")) chunk = std::max(1, std::min(chunk, atoi(ch)));  // tests
      auto need_of = [&](size_t C) {
        return C * (al(4 * N * 8) + al(N * 4)) + al(C * K * g.st[0] * 4) + al(C * g.level_entries * 8) + al(C * K * 4) +
               al(C * 8) + al(C * P * 4) + al(C * sizeof(kf64::EvCfg)) + 4096;
      };
      if (h->swt_bytes < need_of((size_t)chunk)) {
        if (h->swt_scratch) {
          for (auto& b : h->bufs)
            if (b.p == h->swt_scratch) b.p = nullptr;
          (void)hipFree(h->swt_scratch);
          h->swt_scratch = nullptr;
          h->swt_bytes = 0;
        }
        // an allocation that fails halves the scenario chunk until one fits (one scenario at least)
        char* p = nullptr;
        for (;;) {
          const size_t need = need_of((size_t)chunk);
          if (hipMalloc((void**)&p, need) == hipSuccess) {
            h->bufs.push_back({p, need});
            h->swt_scratch = p;
            h->swt_bytes = need;
            break;
          }
          (void)hipGetLastError();
          if (chunk == 1) return ksim_fail(h, KSIM_E_NOMEM, "ksim_sweep: no device memory for one scenario (%zu bytes)", need);
          chunk = (chunk + 1) / 2;
        }
      }
      const size_t C = (size_t)chunk;
      char* q = (char*)h->swt_scratch;
      auto take = [&](size_t b) { char* r = q; q += al(b); return r; };
      KsimTreeSweep sw{};
      sw.count_pods = count;
      sw.rc = (int64_t*)take(C * N * 8); sw.rm = (int64_t*)take(C * N * 8);
      sw.zc = (int64_t*)take(C * N * 8); sw.zm = (int64_t*)take(C * N * 8);
      sw.count = (int32_t*)take(C * N * 4);
      int32_t* leaves = (int32_t*)take(C * K * g.st[0] * 4);
      uint64_t* levels = (uint64_t*)take(C * g.level_entries * 8);
      int32_t* fitc = (int32_t*)take(C * K * 4);
      sw.counter = (uint64_t*)take(C * 8);
      sw.out_node = (int32_t*)take(C * P * 4);
      kf64::EvCfg* dcfg = (kf64::EvCfg*)take(C * sizeof(kf64::EvCfg));
      sw.cfg = dcfg;
      std::vector<kf64::EvCfg> cfgs((size_t)n_scen);
      for (int32_t sidx = 0; sidx < n_scen; ++sidx)
        cfgs[sidx] = kf64::make_evcfg(c.preds, c.no_prio != 0, w3[3 * sidx], w3[3 * sidx + 1], w3[3 * sidx + 2]);
      const int64_t save_first = c.first, save_end = c.end;
      c.first = first;
      c.end = first + count;
      float kms = 0.f, dms = 0.f;
      int32_t err0 = 0;
      HIPCHK(h, hipMemcpy(&err0, c.err, 4, hipMemcpyDeviceToHost));
      for (int32_t s0 = 0; s0 < n_scen; s0 += chunk) {
        sw.nsc = std::min(chunk, n_scen - s0);
        HIPCHK(h, hipMemcpyAsync(dcfg, cfgs.data() + s0, sw.nsc * sizeof(kf64::EvCfg), hipMemcpyHostToDevice, ksim_stream(h)));
        HIPCHK(h, hipEventRecord(h->ev0, ksim_stream(h)));
        hipError_t e = ksim_tree_sweep_init(&c, &sw, ksim_stream(h));
        if (e == hipSuccess) e = ksim_tree_build(&c, &g, h->tclass, h->tcls, leaves, levels, fitc, h->t_y, &sw, ksim_stream(h));
        if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "tree sweep build: %s", hipGetErrorString(e));
        HIPCHK(h, hipEventRecord(h->ev1, ksim_stream(h)));
        e = ksim_tree_launch(&c, &g, h->tclass, h->tcls, leaves, levels, fitc, h->t_y, &sw, ksim_stream(h));
        if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "tree sweep launch: %s", hipGetErrorString(e));
        hipEvent_t ev2 = nullptr;
        HIPCHK(h, hipEventCreate(&ev2));
        HIPCHK(h, hipEventRecord(ev2, ksim_stream(h)));
        HIPCHK(h, hipEventSynchronize(ev2));
        float b_ms = 0.f, r_ms = 0.f;
        HIPCHK(h, hipEventElapsedTime(&b_ms, h->ev0, h->ev1));
        HIPCHK(h, hipEventElapsedTime(&r_ms, h->ev1, ev2));
        (void)hipEventDestroy(ev2);
        kms += r_ms;
        dms += b_ms + r_ms;
        HIPCHK(h, hipMemcpy(out_node + (size_t)s0 * P, sw.out_node, (size_t)sw.nsc * P * 4, hipMemcpyDeviceToHost));
        if (out_counters) HIPCHK(h, hipMemcpy(out_counters + s0, sw.counter, (size_t)sw.nsc * 8, hipMemcpyDeviceToHost));
      }
      c.first = save_first;
      c.end = save_end;
      int32_t err = 0;
      HIPCHK(h, hipMemcpy(&err, c.err, 4, hipMemcpyDeviceToHost));
      if (err != err0) {
        HIPCHK(h, hipMemcpy(c.err, &err0, 4, hipMemcpyHostToDevice));
        return ksim_fail(h, KSIM_E_DEVICE, "tree sweep: device consistency error 0x%x", err & ~err0);
      }
      if (st) {
        memset(st, 0, sizeof *st);
        st->pods = (int64_t)(n_scen * P);
        int64_t b = 0;
        for (size_t k = 0; k < (size_t)n_scen * P; ++k) b += out_node[k] >= 0;
        st->scheduled = b;
        st->node_evals = (int64_t)(n_scen * P) * n;
        st->device_ms = dms;
        st->kernel_ms = kms;
        st->kernel_launches = (n_scen + chunk - 1) / chunk;
        st->mode = KSIM_MODE_TREE;
        st->blocks = chunk;
      }
      return KSIM_OK;
    }
  }
  if (!h->sw_dac) {
    if ((rc = dev_alloc(h, &h->sw_dac, n)) || (rc = dev_alloc(h, &h->sw_dam, n)) || (rc = dev_alloc(h, &h->sw_yc, n)) ||
        (rc = dev_alloc(h, &h->sw_ym, n)))
      return rc;
    hipError_t e = ksim_sweep_prepare(c.alloc_cpu, c.alloc_mem, n, h->sw_dac, h->sw_dam, h->sw_yc, h->sw_ym, ksim_stream(h));
    if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "sweep prepare: %s", hipGetErrorString(e));
  }
  // scratch: [S][n] x (4 float64 + int32), pods, weights, outputs
  const size_t S = (size_t)n_scen, N = (size_t)n, P = (size_t)count;
  auto al = [](size_t b) { return (b + 255) & ~(size_t)255; };
  const size_t b_dyn = al(S * N * 8), b_cnt = al(S * N * 4), b_pod = al(P * sizeof(kf64::FPod)), b_w = al(S * 12),
               b_out = al(S * P * 4), b_ctr = al(S * 8);
  const size_t need = 4 * b_dyn + b_cnt + b_pod + b_w + b_out + b_ctr;
  if (h->sw_scratch_bytes < need) {
    if (h->sw_scratch) {
      for (auto& b : h->bufs)
        if (b.p == h->sw_scratch) b.p = nullptr;
      (void)hipFree(h->sw_scratch);
      h->sw_scratch = nullptr;
      h->sw_scratch_bytes = 0;
    }
    char* p = nullptr;
    if ((rc = dev_alloc(h, &p, need))) return rc;
    h->sw_scratch = p;
    h->sw_scratch_bytes = need;
  }
  char* base = (char*)h->sw_scratch;
  SwArgs a{};
  a.n = n; a.n_pods = (int32_t)count; a.scen0 = 0;
  a.dac = h->sw_dac; a.dam = h->sw_dam; a.yc = h->sw_yc; a.ym = h->sw_ym;
  a.allowed = c.allowed_pods; a.flags = c.flags;
  a.rc = (double*)base; a.rm = (double*)(base + b_dyn); a.zc = (double*)(base + 2 * b_dyn);
  a.zm = (double*)(base + 3 * b_dyn);
  a.count = (int32_t*)(base + 4 * b_dyn);
  char* q = base + 4 * b_dyn + b_cnt;
  a.pods = (const kf64::FPod*)q;
  int32_t* dw = (int32_t*)(q + b_pod);
  a.w = dw;
  a.out_node = (int32_t*)(q + b_pod + b_w);
  a.out_counter = (uint64_t*)(q + b_pod + b_w + b_out);
  a.preds = c.preds; a.no_prio = c.no_prio;
  HIPCHK(h, hipMemcpy(&a.counter0, c.counter, 8, hipMemcpyDeviceToHost));
  HIPCHK(h, hipMemcpyAsync(dw, w3.data(), S * 12, hipMemcpyHostToDevice, ksim_stream(h)));
  hipError_t e = ksim_sweep_launch(c.req_cpu, c.req_mem, c.nz_cpu, c.nz_mem, c.pod_count, c.pods + first,
                                   (void*)a.pods, &a, n_scen, h->ev0, h->ev1, ksim_stream(h));
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_DEVICE, "sweep launch: %s", hipGetErrorString(e));
  HIPCHK(h, hipEventSynchronize(h->ev1));
  float ms = 0.f;
  HIPCHK(h, hipEventElapsedTime(&ms, h->ev0, h->ev1));
  HIPCHK(h, hipMemcpy(out_node, a.out_node, S * P * 4, hipMemcpyDeviceToHost));
  if (out_counters) HIPCHK(h, hipMemcpy(out_counters, a.out_counter, S * 8, hipMemcpyDeviceToHost));
  if (st) {
    memset(st, 0, sizeof *st);
    st->pods = (int64_t)(S * P);
    int64_t b = 0;
    for (size_t k = 0; k < S * P; ++k) b += out_node[k] >= 0;
    st->scheduled = b;
    st->node_evals = (int64_t)(S * P) * n;
    st->device_ms = ms;
    st->kernel_ms = ms;
    st->kernel_launches = 1;
    st->mode = KSIM_MODE_PERSISTENT;
    st->blocks = n_scen;
  }
  return KSIM_OK;
}

int ksim_shard_setup(ksim_handle* h, int32_t rank, int32_t world, int64_t node_base) {
  if (!h) return ksim_fail(h, KSIM_E_INVAL, "ksim_shard_setup: null handle");
  if (world < 1 || world > KSIM_MAX_RANKS || rank < 0 || rank >= world || node_base < 0)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_shard_setup: rank %d of %d out of range", rank, world);
  if (h->shard.xchg) return ksim_fail(h, KSIM_E_STATE, "ksim_shard_setup: already set up");
  HIPCHK(h, hipSetDevice(h->device));
  void* p = nullptr;
  const size_t bytes = ksim_shard_xchg_bytes();
  // fine-grained (uncached) so peers' writes over xGMI are seen by this device's polling loads
  hipError_t e = hipExtMallocWithFlags(&p, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return ksim_fail(h, KSIM_E_NOMEM, "exchange buffer: %s", hipGetErrorString(e));
  HIPCHK(h, hipMemset(p, 0, bytes));
  h->shard.rank = rank;
  h->shard.world = world;
  h->shard.node_base = node_base;
  h->shard.xtag_base = 0;
  h->shard.xchg = (uint64_t*)p;
  {  // start handshake bound (seconds): KSIM_SHARD_START_S, default 120
    const char* e = getenv("KSIM_SHARD_START_S");
    const double sec = e ? atof(e) : 120.0;
    h->shard.start_ticks = (uint64_t)((sec > 2.0 ? sec : 2.0) * 1e8);
  }
  for (auto& q : h->shard.peers) q = nullptr;
  h->shard.peers[rank] = h->shard.xchg;
  return KSIM_OK;
}

int ksim_shard_export(ksim_handle* h, uint8_t* out_handle) {
  if (!h || !out_handle) return ksim_fail(h, KSIM_E_INVAL, "ksim_shard_export: null argument");
  if (!h->shard.xchg) return ksim_fail(h, KSIM_E_STATE, "ksim_shard_export: call ksim_shard_setup first");
  HIPCHK(h, hipSetDevice(h->device));
  hipIpcMemHandle_t m;
  HIPCHK(h, hipIpcGetMemHandle(&m, h->shard.xchg));
  static_assert(sizeof(m) <= KSIM_IPC_HANDLE_BYTES, "IPC handle size");
  memset(out_handle, 0, KSIM_IPC_HANDLE_BYTES);
  memcpy(out_handle, &m, sizeof m);
  return KSIM_OK;
}

int ksim_shard_connect(ksim_handle* h, int32_t peer, const uint8_t* peer_handle) {
  if (!h || !peer_handle) return ksim_fail(h, KSIM_E_INVAL, "ksim_shard_connect: null argument");
  if (!h->shard.xchg) return ksim_fail(h, KSIM_E_STATE, "ksim_shard_connect: call ksim_shard_setup first");
  if (peer < 0 || peer >= h->shard.world || peer == h->shard.rank)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_shard_connect: bad peer %d", peer);
  HIPCHK(h, hipSetDevice(h->device));
  hipIpcMemHandle_t m;
  memcpy(&m, peer_handle, sizeof m);
  void* p = nullptr;
  HIPCHK(h, hipIpcOpenMemHandle(&p, m, hipIpcMemLazyEnablePeerAccess));
  h->ipc_mapped[peer] = p;
  h->shard.peers[peer] = (uint64_t*)p;
  return KSIM_OK;
}

int ksim_shard_connect_local(ksim_handle* h, int32_t peer, ksim_handle* peer_h) {
  if (!h || !peer_h) return ksim_fail(h, KSIM_E_INVAL, "ksim_shard_connect_local: null argument");
  if (!h->shard.xchg || !peer_h->shard.xchg) return ksim_fail(h, KSIM_E_STATE, "ksim_shard_connect_local: set up both first");
  if (peer < 0 || peer >= h->shard.world || peer == h->shard.rank || peer_h->shard.rank != peer)
    return ksim_fail(h, KSIM_E_INVAL, "ksim_shard_connect_local: bad peer %d", peer);
  HIPCHK(h, hipSetDevice(h->device));
  if (peer_h->device != h->device) {
    hipError_t e = hipDeviceEnablePeerAccess(peer_h->device, 0);
    if (e != hipSuccess && e != hipErrorPeerAccessAlreadyEnabled)
      return ksim_fail(h, KSIM_E_DEVICE, "peer access to device %d: %s", peer_h->device, hipGetErrorString(e));
    (void)hipGetLastError();
  }
  h->shard.peers[peer] = peer_h->shard.xchg;
  return KSIM_OK;
}

int ksim_read_nodes(ksim_handle* h, ksim_node_state* o) {
  if (!h || !o) return ksim_fail(h, KSIM_E_INVAL, "ksim_read_nodes: null argument");
  if (!h->have_nodes) return ksim_fail(h, KSIM_E_STATE, "ksim_read_nodes: no node table");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  const KsimCtx& c = h->ctx;
  const size_t n = c.n;
  if (o->req_cpu) HIPCHK(h, hipMemcpy(o->req_cpu, c.req_cpu, n * 8, hipMemcpyDeviceToHost));
  if (o->req_mem) HIPCHK(h, hipMemcpy(o->req_mem, c.req_mem, n * 8, hipMemcpyDeviceToHost));
  if (o->req_gpu) HIPCHK(h, hipMemcpy(o->req_gpu, c.req_gpu, n * 8, hipMemcpyDeviceToHost));
  if (o->req_eph) HIPCHK(h, hipMemcpy(o->req_eph, c.req_eph, n * 8, hipMemcpyDeviceToHost));
  if (o->nz_cpu) HIPCHK(h, hipMemcpy(o->nz_cpu, c.nz_cpu, n * 8, hipMemcpyDeviceToHost));
  if (o->nz_mem) HIPCHK(h, hipMemcpy(o->nz_mem, c.nz_mem, n * 8, hipMemcpyDeviceToHost));
  if (o->pod_count) HIPCHK(h, hipMemcpy(o->pod_count, c.pod_count, n * 4, hipMemcpyDeviceToHost));
  if (o->req_scalar && c.n_scalar)
    HIPCHK(h, hipMemcpy(o->req_scalar, c.req_scalar, (size_t)c.n_scalar * n * 8, hipMemcpyDeviceToHost));
  if (o->ports && c.port_slots) HIPCHK(h, hipMemcpy(o->ports, c.ports, (size_t)c.port_slots * n * 8, hipMemcpyDeviceToHost));
  if (o->port_count) HIPCHK(h, hipMemcpy(o->port_count, c.port_count, n * 4, hipMemcpyDeviceToHost));
  return KSIM_OK;
}

int ksim_get_counter(ksim_handle* h, uint64_t* out) {
  if (!h || !out) return ksim_fail(h, KSIM_E_INVAL, "ksim_get_counter: null argument");
  KsimCtrKeep keep(h);
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  HIPCHK(h, hipMemcpy(out, h->ctx.counter, 8, hipMemcpyDeviceToHost));
  // the resident kernel's last answer and the word it stored when it left must agree
  if (keep.known && *out != keep.v)
    return ksim_fail(h, KSIM_E_DEVICE, "lastNodeIndex %llu on the device, %llu in the resident kernel's last answer",
                     (unsigned long long)*out, (unsigned long long)keep.v);
  return KSIM_OK;
}

int ksim_set_counter(ksim_handle* h, uint64_t v) {
  if (!h) return ksim_fail(h, KSIM_E_INVAL, "ksim_set_counter: null handle");
  HIPCHK(h, hipSetDevice(h->device));
  HIPCHK(h, hipStreamSynchronize(ksim_stream(h)));
  HIPCHK(h, hipMemcpy(h->ctx.counter, &v, 8, hipMemcpyHostToDevice));
  return KSIM_OK;
}

}  // extern "C"
