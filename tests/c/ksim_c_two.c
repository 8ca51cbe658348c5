/*
 * Two handles on one device (plain C, include/ksim.h only): a resident per-pod kernel on handle A
 * beside whole-queue persistent calls on handle B, sequentially and from two threads at once.
 *
 * The resident per-pod kernel (ksim_serve_kernel) keeps its blocks on the device between calls;
 * the persistent batch kernels need every workgroup resident at once (they wait on each other).
 * The library's device gate runs such batch calls with every other handle's resident kernel
 * stopped, and holds the next per-pod call until the batch call has finished.  Checked: every
 * per-pod decision and lastNodeIndex of A against the C oracle step by step, every batch run of B
 * against the oracle's run of the same queue, the final node state of A.
 *
 *   ksim_c_two <a_nodes> <a_steps> <b_nodes> <b_pods> <b_runs>
 * Exit status 0 = pass.  Needs a GPU (tests/test_c_abi.py; KSIM_ONE_WG=0 there, so A's calls take
 * the resident kernel).
 *
 * Reference: Scheduler.scheduleOne (vendor/k8s.io/kubernetes/pkg/scheduler/scheduler.go:431-484)
 * per pod on A; the simulator's sequential queue (pkg/scheduler/simulator.go:108-223) on B.
 */
#include <pthread.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ksim.h"

int ksim_ref_run(const ksim_config* cfg, const ksim_node_table* tab, ksim_node_state* st, const ksim_class_tables* ct,
                 const ksim_pod* pods, const uint64_t* pod_ports, const ksim_scalar_req* pod_scalars, int64_t first,
                 int64_t count, int threads, int32_t* out_node, int32_t* out_reasons, uint64_t* io_counter);

static int fails = 0;
static pthread_mutex_t fail_mu = PTHREAD_MUTEX_INITIALIZER;
#define CHECK(cond, ...)                                  \
  do {                                                    \
    if (!(cond)) {                                        \
      pthread_mutex_lock(&fail_mu);                       \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                       \
      fprintf(stderr, "\n");                              \
      if (++fails > 10) exit(1);                          \
      pthread_mutex_unlock(&fail_mu);                     \
    }                                                     \
  } while (0)
#define KS(h, call)                                                                                   \
  do {                                                                                                \
    int rc_ = (call);                                                                                 \
    if (rc_ != KSIM_OK) {                                                                             \
      fprintf(stderr, "FAIL %s:%d: %s -> %d (%s)\n", __FILE__, __LINE__, #call, rc_, ksim_last_error(h)); \
      exit(1);                                                                                        \
    }                                                                                                 \
  } while (0)

typedef struct {  /* one cluster as SoA host columns (no ports: resource pods only) */
  int64_t n;
  int64_t *ac, *am, *z64, *rc, *rm, *zc, *zm;
  int32_t *allowed, *cnt, *pc, *z32;
  uint32_t* flags;
} Cluster;

static uint64_t rnd_state(uint64_t* s) { /* splitmix64 */
  uint64_t z = (*s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

static void cluster_init(Cluster* c, int64_t n, uint64_t seed) {
  static const int64_t cpus[] = {2000, 4000, 8000}, mems[] = {4, 8, 16};
  c->n = n;
  c->ac = calloc(n, 8); c->am = calloc(n, 8); c->z64 = calloc(n, 8); c->rc = calloc(n, 8); c->rm = calloc(n, 8);
  c->zc = calloc(n, 8); c->zm = calloc(n, 8);
  c->allowed = calloc(n, 4); c->cnt = calloc(n, 4); c->pc = calloc(n, 4); c->z32 = calloc(n, 4); c->flags = calloc(n, 4);
  for (int64_t i = 0; i < n; ++i) {
    c->ac[i] = cpus[rnd_state(&seed) % 3];
    c->am[i] = mems[rnd_state(&seed) % 3] << 30;
    c->allowed[i] = 110;
  }
}

static void cluster_tab(const Cluster* c, ksim_node_table* t, ksim_node_state* st) {
  memset(t, 0, sizeof *t);
  t->n_nodes = c->n; t->port_slots = 0;
  t->alloc_cpu = c->ac; t->alloc_mem = c->am; t->alloc_gpu = c->z64; t->alloc_eph = c->z64;
  t->allowed_pods = c->allowed; t->flags = c->flags; t->label_set = c->z32; t->taint_set = c->z32;
  t->req_cpu = c->rc; t->req_mem = c->rm; t->req_gpu = c->z64; t->req_eph = c->z64;
  t->nz_cpu = c->zc; t->nz_mem = c->zm; t->pod_count = c->cnt; t->port_count = c->pc;
  if (st) {
    memset(st, 0, sizeof *st);
    st->req_cpu = c->rc; st->req_mem = c->rm; st->req_gpu = c->z64; st->req_eph = c->z64;
    st->nz_cpu = c->zc; st->nz_mem = c->zm; st->pod_count = c->cnt; st->port_count = c->pc;
  }
}

static ksim_pod rnd_pod(uint64_t* s) {
  static const int64_t cpus[] = {100, 250, 500, 1000, 2000};
  static const int64_t mems[] = {128, 256, 512, 1024, 2048};
  ksim_pod p;
  memset(&p, 0, sizeof p);
  p.req_cpu = p.add_cpu = p.nz_cpu = cpus[rnd_state(s) % 5];
  p.req_mem = p.add_mem = p.nz_mem = mems[rnd_state(s) % 5] << 20;
  p.flags = KSIM_POD_ANY_REQUEST;
  p.host = -1;
  return p;
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
  cfg.mode = mode;
  cfg.predicates = KSIM_P_CHECK_NODE_CONDITION | KSIM_P_GENERAL;
  cfg.weights[KSIM_W_LEAST_REQUESTED] = 1;
  cfg.weights[KSIM_W_BALANCED] = 1;
  cfg.collect_reasons = 1;
  return cfg;
}

/* ---- handle A: per-pod Schedule + assume, each step against the oracle ---- */
typedef struct {
  ksim_handle* h;
  Cluster host;   /* the oracle's copy, advanced with every decision */
  uint64_t rng, counter;
  int steps_done;
} PerPod;

static void perpod_open(PerPod* a, int64_t n) {
  memset(a, 0, sizeof *a);
  cluster_init(&a->host, n, 7);
  a->rng = 11;
  ksim_config cfg = config(KSIM_MODE_AUTO);
  KS(NULL, ksim_create(&cfg, &a->h));
  ksim_node_table t;
  cluster_tab(&a->host, &t, NULL);
  KS(a->h, ksim_load_nodes(a->h, &t));
  ksim_class_tables ct = one_class();
  KS(a->h, ksim_load_classes(a->h, &ct));
}

static void perpod_steps(PerPod* a, int k) {
  ksim_config cfg = config(KSIM_MODE_AUTO);
  ksim_class_tables ct = one_class();
  for (int s = 0; s < k; ++s) {
    ksim_pod p = rnd_pod(&a->rng);
    ksim_result r;
    KS(a->h, ksim_schedule_one(a->h, &p, NULL, 0, NULL, 0, KSIM_SCHEDULE_ASSUME, &r));
    ksim_node_table t;
    ksim_node_state st;
    cluster_tab(&a->host, &t, &st);
    int32_t want = -2, reasons[KSIM_NREASONS];
    CHECK(ksim_ref_run(&cfg, &t, &st, &ct, &p, NULL, NULL, 0, 1, 1, &want, reasons, &a->counter) == KSIM_OK, "oracle");
    CHECK(r.node == want, "A step %d: node %d, oracle %d", a->steps_done, r.node, want);
    CHECK(r.last_node_index == a->counter, "A step %d: lastNodeIndex %llu, oracle %llu", a->steps_done,
          (unsigned long long)r.last_node_index, (unsigned long long)a->counter);
    a->steps_done++;
  }
}

static void perpod_close(PerPod* a) {
  static int64_t rc_[1 << 16], rm_[1 << 16];
  static int32_t cnt_[1 << 16];
  ksim_node_state o;
  memset(&o, 0, sizeof o);
  o.req_cpu = rc_; o.req_mem = rm_; o.pod_count = cnt_;
  KS(a->h, ksim_read_nodes(a->h, &o));
  int bad = 0;
  for (int64_t i = 0; i < a->host.n; ++i) bad += rc_[i] != a->host.rc[i] || rm_[i] != a->host.rm[i] || cnt_[i] != a->host.cnt[i];
  CHECK(bad == 0, "A final state: %d rows differ", bad);
  uint64_t dc = 0;
  KS(a->h, ksim_get_counter(a->h, &dc));
  CHECK(dc == a->counter, "A final lastNodeIndex %llu vs %llu", (unsigned long long)dc, (unsigned long long)a->counter);
  ksim_destroy(a->h);
}

/* ---- handle B: the whole queue in one persistent call, against the oracle's run ---- */
typedef struct {
  int64_t n;
  int npods;
  ksim_pod* q;
  int32_t* want;
  uint64_t want_ctr;
} Batch;

static void batch_prepare(Batch* b, int64_t n, int npods) {
  b->n = n;
  b->npods = npods;
  uint64_t s = 99;
  b->q = calloc(npods, sizeof(ksim_pod));
  for (int k = 0; k < npods; ++k) b->q[k] = rnd_pod(&s);
  b->want = calloc(npods, 4);
  Cluster c;
  cluster_init(&c, n, 5);
  ksim_node_table t;
  ksim_node_state st;
  cluster_tab(&c, &t, &st);
  ksim_config cfg = config(KSIM_MODE_AUTO);
  ksim_class_tables ct = one_class();
  int32_t* reasons = calloc((size_t)npods * KSIM_NREASONS, 4);
  b->want_ctr = 0;
  CHECK(ksim_ref_run(&cfg, &t, &st, &ct, b->q, NULL, NULL, 0, npods, 8, b->want, reasons, &b->want_ctr) == KSIM_OK, "oracle B");
  free(reasons);
}

static void batch_run(const Batch* b, int run) {
  Cluster c;
  cluster_init(&c, b->n, 5);
  ksim_config cfg = config(KSIM_MODE_AUTO);
  ksim_handle* h = NULL;
  KS(NULL, ksim_create(&cfg, &h));
  ksim_node_table t;
  cluster_tab(&c, &t, NULL);
  KS(h, ksim_load_nodes(h, &t));
  ksim_class_tables ct = one_class();
  KS(h, ksim_load_classes(h, &ct));
  KS(h, ksim_load_pods(h, b->q, b->npods, NULL, 0, NULL, 0));
  int32_t* got = calloc(b->npods, 4);
  ksim_stats st;
  KS(h, ksim_schedule(h, 0, b->npods, got, NULL, &st));
  int diff = 0;
  for (int k = 0; k < b->npods; ++k) diff += got[k] != b->want[k];
  uint64_t ctr = 0;
  KS(h, ksim_get_counter(h, &ctr));
  CHECK(diff == 0, "B run %d (mode %d): %d of %d placements differ", run, st.mode, diff, b->npods);
  CHECK(ctr == b->want_ctr, "B run %d: lastNodeIndex %llu vs %llu", run, (unsigned long long)ctr, (unsigned long long)b->want_ctr);
  if (run == 0) printf("B: %d pods on %lld nodes, kernel mode %d\n", b->npods, (long long)b->n, st.mode);
  free(got);
  ksim_destroy(h);
}

typedef struct {
  PerPod* a;
  int steps;
} AThread;
static void* a_thread(void* arg) {
  AThread* x = (AThread*)arg;
  perpod_steps(x->a, x->steps);
  return NULL;
}

int main(int argc, char** argv) {
  const int64_t a_nodes = argc > 1 ? atoll(argv[1]) : 5000;
  const int a_steps = argc > 2 ? atoi(argv[2]) : 2000;
  const int64_t b_nodes = argc > 3 ? atoll(argv[3]) : 20000;
  const int b_pods = argc > 4 ? atoi(argv[4]) : 4000;
  const int b_runs = argc > 5 ? atoi(argv[5]) : 4;
  if (a_nodes < 1 || a_nodes > (1 << 16) || a_steps < 1 || b_nodes < 1 || b_pods < 1 || b_runs < 1) return 2;
  Batch b;
  batch_prepare(&b, b_nodes, b_pods);
  PerPod a;
  perpod_open(&a, a_nodes);
  /* 1. sequential: A's resident kernel is live when B's batch call starts */
  perpod_steps(&a, a_steps / 4);
  batch_run(&b, 0);
  perpod_steps(&a, a_steps / 4);
  /* 2. concurrent: A's per-pod calls on one thread while B's batch calls run on another */
  pthread_t th;
  AThread x = {&a, a_steps / 2};
  if (pthread_create(&th, NULL, a_thread, &x) != 0) return 2;
  for (int r = 1; r < b_runs; ++r) batch_run(&b, r);
  pthread_join(th, NULL);
  perpod_close(&a);
  printf("two handles: A %d per-pod steps on %lld nodes, B %d batch runs\n", a.steps_done, (long long)a_nodes, b_runs);
  if (fails) {
    printf("FAILED (%d checks)\n", fails);
    return 1;
  }
  printf("PASS\n");
  return 0;
}
