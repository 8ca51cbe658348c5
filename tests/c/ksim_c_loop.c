/*
 * Plain-C drop-in test of libksim.so — what a cgo binding sees: only include/ksim.h, only C.
 *
 * It drives a scheduleOne-style loop (vendor/k8s.io/kubernetes/pkg/scheduler/scheduler.go:431-484:
 * Schedule → assume) one pod at a time through ksim_schedule_one, interleaved with the cache
 * events the informers deliver (factory/factory.go:596,695,740,755,841 → schedulercache/cache.go
 * AddPod / RemovePod / AddNode / UpdateNode / RemoveNode), and checks every decision against the
 * C oracle (oracle/cpu_ref.c, ksim_ref_run on the same node table kept on the host), plus:
 *   1. batch parity — one queue through ksim_schedule (persistent / auto) and the same pods
 *      one at a time through ksim_schedule_one give identical placements and lastNodeIndex;
 *   2. the final device node state equals the host copy column by column.
 * Exit status 0 = pass; prints one summary line.  Needs a GPU (run by tests/test_c_abi.py).
 *
 *   ksim_c_loop <nodes> <steps> [gap_ms gap_every [adapter]]
 * gap_ms / gap_every: sleep gap_ms before every gap_every-th step of the event loop (a scheduler
 * whose pods arrive sporadically: the resident per-pod kernel leaves by its idle vote and is
 * relaunched, or a message meets a grid on its way out).
 * adapter = 1: every Schedule is the cgo adapter's pattern — KSIM_SCHEDULE_ONLY, then (8 in 10)
 * ksim_pod_add onto the chosen node (Scheduler.assume), (1 in 10) onto another node (the binding
 * landed elsewhere), or (1 in 10) nothing (the pod is dropped) — so the resident kernel's
 * tentative commits are confirmed, undone by a different assume, or undone by the next event.
 *
 * Build: tests/c/Makefile (gcc, links libksim.so and the oracle's libksim_ref.so).
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ksim.h"

/* oracle/cpu_ref.c (test infrastructure) */
int ksim_ref_run(const ksim_config* cfg, const ksim_node_table* tab, ksim_node_state* st, const ksim_class_tables* ct,
                 const ksim_pod* pods, const uint64_t* pod_ports, const ksim_scalar_req* pod_scalars, int64_t first,
                 int64_t count, int threads, int32_t* out_node, int32_t* out_reasons, uint64_t* io_counter);

#define MAXN 2048
#define HP 8 /* host-side port slots per node */

typedef struct {
  char name[24];
  int64_t ac, am;
  int32_t allowed;
  uint32_t flags;
  int64_t rc, rm, zc, zm;
  int32_t cnt, pc;
  uint64_t ports[HP];
} HNode;

typedef struct {
  ksim_pod pod;
  uint64_t port;
  char node[24];
} Placed;

static uint64_t rng_s = 0x9E3779B97F4A7C15ull;
static uint64_t rnd(void) { /* splitmix64 */
  uint64_t z = (rng_s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static int64_t pick(const int64_t* v, int n) { return v[rnd() % (uint64_t)n]; }

static HNode nodes[MAXN];
static int64_t n_nodes = 0;
static int fails = 0;

#define CHECK(cond, ...)                            \
  do {                                              \
    if (!(cond)) {                                  \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                 \
      fprintf(stderr, "\n");                        \
      if (++fails > 10) exit(1);                    \
    }                                               \
  } while (0)

#define KS(h, call)                                                                   \
  do {                                                                                \
    int rc_ = (call);                                                                 \
    if (rc_ != KSIM_OK) {                                                             \
      fprintf(stderr, "FAIL %s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_, ksim_last_error(h)); \
      exit(1);                                                                        \
    }                                                                                 \
  } while (0)

/* bytewise name rank (Go string <): the node table's order */
static int64_t rank_of(const char* name) {
  int64_t lo = 0, hi = n_nodes;
  while (lo < hi) {
    int64_t mid = (lo + hi) / 2;
    if (strcmp(nodes[mid].name, name) < 0) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

static HNode rnd_node(int id) {
  static const int64_t cpus[] = {2000, 4000, 8000}, mems[] = {4, 8, 16};
  HNode x;
  memset(&x, 0, sizeof x);
  snprintf(x.name, sizeof x.name, "node-%d", id);
  x.ac = pick(cpus, 3);
  x.am = pick(mems, 3) << 30;
  x.allowed = (rnd() % 10) ? 110 : 6;
  x.flags = (rnd() % 20) ? 0u : KSIM_N_NOT_READY;
  return x;
}

static ksim_pod rnd_pod(uint64_t* port) {
  static const int64_t cpus[] = {100, 250, 500, 1000, 2000};
  static const int64_t mems[] = {128, 256, 512, 1024, 2048};
  static const int64_t hports[] = {8080, 9090, 10250};
  ksim_pod p;
  memset(&p, 0, sizeof p);
  p.req_cpu = p.add_cpu = p.nz_cpu = pick(cpus, 5);
  p.req_mem = p.add_mem = p.nz_mem = pick(mems, 5) << 20;
  p.flags = KSIM_POD_ANY_REQUEST;
  p.host = -1;
  *port = 0;
  if (rnd() % 4 == 0) {
    *port = KSIM_PORT_KEY(rnd() % 2, 0, pick(hports, 3));
    p.port_cnt = 1;
  }
  return p;
}

static ksim_node_row row_of(const HNode* x) {
  ksim_node_row r;
  memset(&r, 0, sizeof r);
  r.alloc_cpu = x->ac;
  r.alloc_mem = x->am;
  r.allowed_pods = x->allowed;
  r.flags = x->flags;
  r.req_cpu = x->rc; r.req_mem = x->rm; r.nz_cpu = x->zc; r.nz_mem = x->zm;
  r.pod_count = x->cnt;
  r.port_count = x->pc;
  r.ports = x->ports;
  return r;
}

/* SoA image of the host nodes for the oracle / the initial load */
typedef struct {
  int64_t ac[MAXN], am[MAXN], zero64[MAXN], rc[MAXN], rm[MAXN], zc[MAXN], zm[MAXN];
  int32_t allowed[MAXN], cnt[MAXN], pc[MAXN], zero32[MAXN];
  uint32_t flags[MAXN];
  uint64_t ports[HP * MAXN];
} Soa;
static Soa soa;

static void to_soa(ksim_node_table* t, ksim_node_state* st, int32_t slots) {
  const int64_t n = n_nodes;
  memset(&soa.zero64, 0, sizeof soa.zero64);
  memset(&soa.zero32, 0, sizeof soa.zero32);
  for (int64_t i = 0; i < n; ++i) {
    const HNode* x = &nodes[i];
    soa.ac[i] = x->ac; soa.am[i] = x->am; soa.allowed[i] = x->allowed; soa.flags[i] = x->flags;
    soa.rc[i] = x->rc; soa.rm[i] = x->rm; soa.zc[i] = x->zc; soa.zm[i] = x->zm; soa.cnt[i] = x->cnt; soa.pc[i] = x->pc;
    for (int s = 0; s < slots; ++s) soa.ports[(int64_t)s * n + i] = s < x->pc ? x->ports[s] : 0;
  }
  memset(t, 0, sizeof *t);
  t->n_nodes = n; t->n_scalar = 0; t->port_slots = slots;
  t->alloc_cpu = soa.ac; t->alloc_mem = soa.am; t->alloc_gpu = soa.zero64; t->alloc_eph = soa.zero64;
  t->allowed_pods = soa.allowed; t->flags = soa.flags; t->label_set = soa.zero32; t->taint_set = soa.zero32;
  t->req_cpu = soa.rc; t->req_mem = soa.rm; t->req_gpu = soa.zero64; t->req_eph = soa.zero64;
  t->nz_cpu = soa.zc; t->nz_mem = soa.zm; t->pod_count = soa.cnt; t->ports = soa.ports; t->port_count = soa.pc;
  if (st) {
    memset(st, 0, sizeof *st);
    st->req_cpu = soa.rc; st->req_mem = soa.rm; st->req_gpu = soa.zero64; st->req_eph = soa.zero64;
    st->nz_cpu = soa.zc; st->nz_mem = soa.zm; st->pod_count = soa.cnt; st->ports = soa.ports; st->port_count = soa.pc;
  }
}

static void from_soa(void) {
  const int64_t n = n_nodes;
  for (int64_t i = 0; i < n; ++i) {
    HNode* x = &nodes[i];
    x->rc = soa.rc[i]; x->rm = soa.rm[i]; x->zc = soa.zc[i]; x->zm = soa.zm[i]; x->cnt = soa.cnt[i]; x->pc = soa.pc[i];
    for (int s = 0; s < HP; ++s) x->ports[s] = s < x->pc ? soa.ports[(int64_t)s * n + i] : 0;
  }
}

/* NodeInfo.AddPod / RemovePod on the host copy (node_info.go:318-390) */
static void host_add(HNode* x, const ksim_pod* p, uint64_t port) {
  x->rc += p->add_cpu; x->rm += p->add_mem; x->zc += p->nz_cpu; x->zm += p->nz_mem; x->cnt += 1;
  if (p->port_cnt) {
    for (int s = 0; s < x->pc; ++s)
      if (x->ports[s] == port) return;
    if (x->pc < HP) x->ports[x->pc++] = port;
  }
}
static void host_remove(HNode* x, const ksim_pod* p, uint64_t port) {
  x->rc -= p->add_cpu; x->rm -= p->add_mem; x->zc -= p->nz_cpu; x->zm -= p->nz_mem; x->cnt -= 1;
  if (p->port_cnt) {
    for (int s = 0; s < x->pc; ++s)
      if (x->ports[s] == port) { x->ports[s] = x->ports[x->pc - 1]; x->ports[--x->pc] = 0; return; }
  }
}

static ksim_class_tables one_class(void) {
  static uint32_t ok = 1u;
  static uint8_t zero8 = 0;
  static int32_t one = 1;
  static int64_t vals[KSIM_MAX_RCLASS];
  ksim_class_tables ct;
  memset(&ct, 0, sizeof ct);
  ct.n_classes = 1; ct.n_label_sets = 1; ct.n_taint_sets = 1;
  ct.sel_ok = &ok; ct.taint_ok = &ok; ct.noexec_ok = &ok; ct.tt_class = &zero8; ct.na_class = &zero8;
  ct.n_tt = &one; ct.n_na = &one; ct.tt_val = vals; ct.na_val = vals;
  return ct;
}

static ksim_config config(int mode) {
  ksim_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.device = 0;
  cfg.mode = mode;
  cfg.predicates = KSIM_P_CHECK_NODE_CONDITION | KSIM_P_GENERAL;
  cfg.weights[KSIM_W_LEAST_REQUESTED] = 1;
  cfg.weights[KSIM_W_BALANCED] = 1;
  cfg.collect_reasons = 1;
  return cfg;
}

static void insert_node(const HNode* x) {
  const int64_t r = rank_of(x->name);
  memmove(&nodes[r + 1], &nodes[r], (size_t)(n_nodes - r) * sizeof(HNode));
  nodes[r] = *x;
  ++n_nodes;
}

/* ---- 1. batch vs one-at-a-time on the initial cluster ---- */
static void batch_parity(int n0, unsigned npods) {
  ksim_class_tables ct = one_class();
  ksim_pod* q = (ksim_pod*)calloc(npods, sizeof(ksim_pod));
  uint64_t* qp = (uint64_t*)calloc(npods, sizeof(uint64_t));
  int32_t nports = 0;
  for (unsigned k = 0; k < npods; ++k) {
    uint64_t port;
    q[k] = rnd_pod(&port);
    if (q[k].port_cnt) { q[k].port_off = nports; qp[nports++] = port; }
  }
  ksim_node_table t;
  int32_t* a = (int32_t*)malloc(sizeof(int32_t) * npods);
  int32_t* b = (int32_t*)malloc(sizeof(int32_t) * npods);
  int32_t* c = (int32_t*)malloc(sizeof(int32_t) * npods);
  uint64_t ca = 0, cb = 0, cc = 0;
  {  /* batch: the loaded queue through ksim_schedule */
    ksim_config cfg = config(KSIM_MODE_AUTO);
    ksim_handle* h = NULL;
    KS(NULL, ksim_create(&cfg, &h));
    to_soa(&t, NULL, HP);
    KS(h, ksim_load_nodes(h, &t));
    KS(h, ksim_load_classes(h, &ct));
    KS(h, ksim_load_pods(h, q, npods, qp, nports, NULL, 0));
    ksim_stats st;
    KS(h, ksim_schedule(h, 0, npods, a, NULL, &st));
    KS(h, ksim_get_counter(h, &ca));
    ksim_destroy(h);
  }
  {  /* one pod per call, the same pods as descriptors */
    ksim_config cfg = config(KSIM_MODE_AUTO);
    ksim_handle* h = NULL;
    KS(NULL, ksim_create(&cfg, &h));
    to_soa(&t, NULL, 1);  /* a single port slot: the library grows it on demand */
    KS(h, ksim_load_nodes(h, &t));
    KS(h, ksim_load_classes(h, &ct));
    for (unsigned k = 0; k < npods; ++k) {
      ksim_result r;
      KS(h, ksim_schedule_one(h, &q[k], qp, nports, NULL, 0, KSIM_SCHEDULE_ASSUME, &r));
      b[k] = r.node;
      cb = r.last_node_index;
    }
    ksim_destroy(h);
  }
  {  /* the C oracle */
    ksim_config cfg = config(KSIM_MODE_AUTO);
    ksim_node_state st;
    to_soa(&t, &st, HP);
    int32_t* reasons = (int32_t*)calloc((size_t)npods * KSIM_NREASONS, sizeof(int32_t));
    int rc = ksim_ref_run(&cfg, &t, &st, &ct, q, qp, NULL, 0, npods, 1, c, reasons, &cc);
    CHECK(rc == KSIM_OK, "oracle run %d", rc);
    free(reasons);
  }
  int diff = 0, bound = 0;
  for (unsigned k = 0; k < npods; ++k) {
    diff += (a[k] != b[k]) || (a[k] != c[k]);
    bound += a[k] >= 0;
  }
  CHECK(diff == 0, "batch parity: %d of %u placements differ", diff, npods);
  CHECK(ca == cb && ca == cc, "batch parity: lastNodeIndex %llu / %llu / %llu", (unsigned long long)ca,
        (unsigned long long)cb, (unsigned long long)cc);
  printf("batch parity: %u pods (%d bound) on %d nodes, lastNodeIndex %llu\n", npods, bound, n0, (unsigned long long)ca);
  free(q); free(qp); free(a); free(b); free(c);
}

/* ---- 2. scheduleOne loop with cache events vs the oracle ---- */
static int gap_ms = 0, gap_every = 0, adapter = 0;

static void event_loop(int steps) {
  ksim_class_tables ct = one_class();
  ksim_config cfg = config(KSIM_MODE_AUTO);
  ksim_handle* h = NULL;
  KS(NULL, ksim_create(&cfg, &h));
  ksim_node_table t;
  to_soa(&t, NULL, 1);
  KS(h, ksim_load_nodes(h, &t));
  KS(h, ksim_load_classes(h, &ct));
  Placed* placed = (Placed*)calloc((size_t)steps + 1, sizeof(Placed));
  int np = 0, next_id = 100000;
  uint64_t counter = 0;
  int n_sched = 0, n_fit_err = 0, n_add = 0, n_rm = 0, n_nadd = 0, n_nupd = 0, n_nrm = 0;
  for (int step = 0; step < steps; ++step) {
    if (gap_every > 0 && gap_ms > 0 && step % gap_every == gap_every - 1) {
      struct timespec ts = {gap_ms / 1000, (long)(gap_ms % 1000) * 1000000L};
      nanosleep(&ts, NULL);
    }
    const uint64_t r = rnd() % 100;
    if ((r < 70 || n_nodes == 0) && adapter) {  /* Schedule (decide only), then the adapter's assume */
      uint64_t port;
      ksim_pod p = rnd_pod(&port);
      ksim_result res;
      int rc = ksim_schedule_one(h, &p, &port, p.port_cnt, NULL, 0, KSIM_SCHEDULE_ONLY, &res);
      if (n_nodes == 0) {
        CHECK(rc == KSIM_E_NO_NODES, "empty table: %d", rc);
        continue;
      }
      KS(h, rc);
      ksim_node_state st;
      to_soa(&t, &st, HP);
      int32_t want = -2, reasons[KSIM_NREASONS];
      CHECK(ksim_ref_run(&cfg, &t, &st, &ct, &p, &port, NULL, 0, 1, 1, &want, reasons, &counter) == KSIM_OK, "oracle");
      /* (no from_soa: the oracle's commit is not the cache's until the assume below) */
      ++n_sched;
      CHECK(res.node == want, "step %d: node %d, oracle %d", step, res.node, want);
      CHECK(res.last_node_index == counter, "step %d: lastNodeIndex %llu, oracle %llu", step,
            (unsigned long long)res.last_node_index, (unsigned long long)counter);
      if (want < 0) {
        ++n_fit_err;
        CHECK(memcmp(res.reasons, reasons, sizeof reasons) == 0, "step %d: FitError histogram differs", step);
        continue;
      }
      const uint64_t u = rnd() % 10;
      const int64_t w = u < 8 ? want : (u < 9 ? (int64_t)(rnd() % (uint64_t)n_nodes) : -1);
      if (w >= 0) {
        KS(h, ksim_pod_add(h, w, &p, &port, p.port_cnt, NULL, 0));
        host_add(&nodes[w], &p, port);
        placed[np].pod = p; placed[np].port = port;
        strcpy(placed[np].node, nodes[w].name);
        ++np;
        ++n_add;
      }
    } else if (r < 70 || n_nodes == 0) {  /* Schedule + assume */
      uint64_t port;
      ksim_pod p = rnd_pod(&port);
      ksim_result res;
      int rc = ksim_schedule_one(h, &p, &port, p.port_cnt, NULL, 0, KSIM_SCHEDULE_ASSUME, &res);
      if (n_nodes == 0) {
        CHECK(rc == KSIM_E_NO_NODES, "empty table: %d", rc);
        continue;
      }
      KS(h, rc);
      ksim_node_state st;
      to_soa(&t, &st, HP);
      int32_t want = -2, reasons[KSIM_NREASONS];
      CHECK(ksim_ref_run(&cfg, &t, &st, &ct, &p, &port, NULL, 0, 1, 1, &want, reasons, &counter) == KSIM_OK, "oracle");
      from_soa();
      ++n_sched;
      CHECK(res.node == want, "step %d: node %d, oracle %d", step, res.node, want);
      CHECK(res.last_node_index == counter, "step %d: lastNodeIndex %llu, oracle %llu", step,
            (unsigned long long)res.last_node_index, (unsigned long long)counter);
      if (want < 0) {
        ++n_fit_err;
        CHECK(memcmp(res.reasons, reasons, sizeof reasons) == 0, "step %d: FitError histogram differs", step);
      } else if (want >= 0 && res.node == want) {
        placed[np].pod = p; placed[np].port = port;
        strcpy(placed[np].node, nodes[want].name);
        ++np;
      }
    } else if (r < 78 && np > 0) {  /* cache.RemovePod */
      const int k = (int)(rnd() % (uint64_t)np);
      const int64_t w = rank_of(placed[k].node);
      KS(h, ksim_pod_remove(h, w, &placed[k].pod, &placed[k].port, placed[k].pod.port_cnt, NULL, 0));
      host_remove(&nodes[w], &placed[k].pod, placed[k].port);
      placed[k] = placed[--np];
      ++n_rm;
    } else if (r < 85) {  /* cache.AddPod of a pod bound elsewhere (sometimes a burst: an informer
                             resync; the resident per-pod kernel answers each from one block) */
      const int burst = rnd() % 4 == 0 ? 12 : 1;
      for (int b = 0; b < burst && np < steps; ++b) {
        uint64_t port;
        ksim_pod p = rnd_pod(&port);
        const int64_t w = (int64_t)(rnd() % (uint64_t)n_nodes);
        KS(h, ksim_pod_add(h, w, &p, &port, p.port_cnt, NULL, 0));
        host_add(&nodes[w], &p, port);
        placed[np].pod = p; placed[np].port = port;
        strcpy(placed[np].node, nodes[w].name);
        ++np;
        ++n_add;
      }
    } else if (r < 91 && n_nodes < MAXN - 1) {  /* cache.AddNode */
      HNode x = rnd_node(next_id++ % 997 * 1009 % 100003);
      if (rank_of(x.name) < n_nodes && strcmp(nodes[rank_of(x.name)].name, x.name) == 0) continue;
      ksim_node_row row = row_of(&x);
      KS(h, ksim_node_add(h, rank_of(x.name), &row));
      insert_node(&x);
      ++n_nadd;
    } else if (r < 96) {  /* cache.UpdateNode → SetNode (static columns) */
      const int64_t w = (int64_t)(rnd() % (uint64_t)n_nodes);
      HNode x = nodes[w];
      static const int64_t cpus[] = {1000, 3000, 6000};
      if (rnd() % 2) x.ac = pick(cpus, 3);
      else x.flags ^= KSIM_N_NOT_READY;
      ksim_node_row row = row_of(&x);
      KS(h, ksim_node_update(h, w, &row));
      nodes[w].ac = x.ac;
      nodes[w].flags = x.flags;
      ++n_nupd;
    } else if (n_nodes > 1) {  /* cache.RemoveNode (its pods stay out of the listed set) */
      const int64_t w = (int64_t)(rnd() % (uint64_t)n_nodes);
      KS(h, ksim_node_remove(h, w));
      for (int k = 0; k < np;)
        if (strcmp(placed[k].node, nodes[w].name) == 0) placed[k] = placed[--np];
        else ++k;
      memmove(&nodes[w], &nodes[w + 1], (size_t)(n_nodes - w - 1) * sizeof(HNode));
      --n_nodes;
      ++n_nrm;
    }
  }
  /* final device state == host copy */
  int64_t n_dev = -1;
  KS(h, ksim_node_count(h, &n_dev));
  CHECK(n_dev == n_nodes, "node count %lld vs %lld", (long long)n_dev, (long long)n_nodes);
  static int64_t rc_[MAXN], rm_[MAXN], zc_[MAXN], zm_[MAXN];
  static int32_t cnt_[MAXN], pc_[MAXN];
  ksim_node_state o;
  memset(&o, 0, sizeof o);
  o.req_cpu = rc_; o.req_mem = rm_; o.nz_cpu = zc_; o.nz_mem = zm_; o.pod_count = cnt_; o.port_count = pc_;
  KS(h, ksim_read_nodes(h, &o));
  int bad = 0;
  for (int64_t i = 0; i < n_nodes; ++i)
    bad += rc_[i] != nodes[i].rc || rm_[i] != nodes[i].rm || zc_[i] != nodes[i].zc || zm_[i] != nodes[i].zm ||
           cnt_[i] != nodes[i].cnt || pc_[i] != nodes[i].pc;
  CHECK(bad == 0, "final state: %d of %lld rows differ", bad, (long long)n_nodes);
  uint64_t dc = 0;
  KS(h, ksim_get_counter(h, &dc));
  CHECK(dc == counter, "final lastNodeIndex %llu vs %llu", (unsigned long long)dc, (unsigned long long)counter);
  printf("event loop: %d steps, %d schedules (%d FitErrors), pod add %d / remove %d, node add %d / update %d / remove %d, "
         "%lld nodes at the end, lastNodeIndex %llu\n", steps, n_sched, n_fit_err, n_add, n_rm, n_nadd, n_nupd, n_nrm,
         (long long)n_nodes, (unsigned long long)counter);
  free(placed);
  ksim_destroy(h);
}

int main(int argc, char** argv) {
  int n0 = argc > 1 ? atoi(argv[1]) : 300;
  int steps = argc > 2 ? atoi(argv[2]) : 3000;
  if (n0 < 1 || n0 > MAXN / 2) n0 = 300;
  if (steps < 1 || steps > 1000000) steps = 3000;
  if (argc > 4) {
    gap_ms = atoi(argv[3]);
    gap_every = atoi(argv[4]);
  }
  if (argc > 5) adapter = atoi(argv[5]);
  if (ksim_abi_version() != KSIM_ABI_VERSION) {
    fprintf(stderr, "FAIL: ABI %d vs header %d\n", ksim_abi_version(), KSIM_ABI_VERSION);
    return 1;
  }
  for (int i = 0; i < n0; ++i) {
    HNode x = rnd_node(i);
    insert_node(&x);
  }
  batch_parity(n0, 4u * (unsigned)n0);
  event_loop(steps);
  if (fails) {
    printf("FAILED (%d checks)\n", fails);
    return 1;
  }
  printf("PASS\n");
  return 0;
}
