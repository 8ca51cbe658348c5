/*
 * Plain-C test of the self-contained boundary: Kubernetes fields in, placements out, through
 * include/ksim_k8s.h alone — what a cgo adapter does with v1 objects, with no Python and no
 * re-implemented scheduling rule on the caller's side.
 *
 * A synthetic cluster (nodes with zone / tier / hostname labels, NoSchedule and PreferNoSchedule
 * taints, NotReady nodes; pods with nodeSelectors, tolerations, host ports, app labels selected by
 * per-app services (SelectorSpread), required hostname anti-affinity and GCE PD / EBS volumes; running
 * pods bound to nodes) is flattened into ksim_k8s_* structs and
 *   1. scheduled as one queue (ksim_k8s_build → ksim_k8s_open → ksim_schedule) and checked pod by
 *      pod against the C oracle (oracle/cpu_ref.c ksim_ref_run_ex) run on the tables the front end
 *      built (ksim_k8s_tables): placements, FitError histograms, lastNodeIndex;
 *   2. scheduled again one pod at a time on a second snapshot without a queue — scheduleOne
 *      (pkg/scheduler/scheduler.go:431-484): ksim_k8s_describe (the pod's class, identity,
 *      affinity and volume classes interned, tables reloaded when new) → ksim_schedule_one with
 *      assume → ksim_k8s_bind — and checked against the queue run.
 * Exit status 0 = pass; prints one summary line.  Needs a GPU (tests/test_c_abi.py).
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ksim_k8s.h"

/* oracle/cpu_ref.c (test infrastructure) */
typedef struct {
  int32_t* cnt;
  int64_t* carried;
  uint64_t* vslots;
  int32_t* vcount;
  uint32_t* svc_conflict;
  int32_t svc_err;
  int32_t pad;
} ksim_ref_extra;
int ksim_ref_run_ex(const ksim_config* cfg, const ksim_node_table* tab, ksim_node_state* st, const ksim_class_tables* ct,
                    const ksim_affinity_tables* at, const ksim_volume_tables* vt, ksim_ref_extra* xs,
                    const ksim_pod* pods, const uint64_t* pod_ports, const ksim_scalar_req* pod_scalars, int64_t first,
                    int64_t count, int threads, int32_t* out_node, int32_t* out_reasons, uint64_t* io_counter);

static uint64_t rng_s = 0x2545F4914F6CDD1Dull;
static uint64_t rnd(void) {
  uint64_t z = (rng_s += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static double frand(void) { return (double)(rnd() >> 11) / 9007199254740992.0; }

static int fails = 0;
#define CHECK(cond, ...)                              \
  do {                                                \
    if (!(cond)) {                                    \
      if (fails++ < 10) {                             \
        fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
        fprintf(stderr, __VA_ARGS__);                 \
        fprintf(stderr, "\n");                        \
      }                                               \
    }                                                 \
  } while (0)
#define OK(x)                                                              \
  do {                                                                     \
    int rc_ = (x);                                                         \
    if (rc_) {                                                             \
      fprintf(stderr, "%s failed: %d\n", #x, rc_);                         \
      exit(2);                                                             \
    }                                                                      \
  } while (0)

/* string pool: everything the flattened objects point at lives until exit */
static char* S(const char* fmt, ...) __attribute__((format(printf, 1, 2)));
#include <stdarg.h>
static char* S(const char* fmt, ...) {
  char buf[128];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  char* p = malloc(strlen(buf) + 1);
  strcpy(p, buf);
  return p;
}

#define NAPP 12
typedef struct {
  ksim_k8s_node n;
  ksim_k8s_kv labels[3];
  ksim_k8s_taint taint;
  ksim_k8s_condition cond;
} NodeObj;

typedef struct {
  ksim_k8s_pod p;
  ksim_k8s_kv label;
  ksim_k8s_container c;
  ksim_k8s_port port;
  ksim_k8s_kv nsel;
  ksim_k8s_toleration tol;
  ksim_k8s_pod_term anti;
  ksim_k8s_kv anti_ml;
  ksim_k8s_volume vol;
  ksim_k8s_label_selector spread;
  ksim_k8s_kv spread_ml;
  int32_t spread_set;
} PodObj;

static void make_node(NodeObj* o, int i) {
  memset(o, 0, sizeof *o);
  const char* name = S("node-%04d", (int)((i * 7919) % 100000));
  int nl = 0;
  o->labels[nl++] = (ksim_k8s_kv){"kubernetes.io/hostname", name};
  o->labels[nl++] = (ksim_k8s_kv){"tier", S("%c", "abc"[rnd() % 3])};
  if (frand() < 0.7) o->labels[nl++] = (ksim_k8s_kv){"failure-domain.beta.kubernetes.io/zone", S("z%d", (int)(rnd() % 4))};
  o->n.name = name;
  o->n.n_labels = nl;
  o->n.labels = o->labels;
  const double r = frand();
  if (r < 0.1) o->taint = (ksim_k8s_taint){"dedicated", "gpu", "NoSchedule"};
  else if (r < 0.2) o->taint = (ksim_k8s_taint){"spot", "true", "PreferNoSchedule"};
  o->n.n_taints = r < 0.2 ? 1 : 0;
  o->n.taints = &o->taint;
  o->cond = (ksim_k8s_condition){"Ready", frand() < 0.01 ? "False" : "True"};
  o->n.n_conditions = 1;
  o->n.conditions = &o->cond;
  static const int64_t cpus[] = {8000, 16000, 32000, 64000};
  static const int64_t mems[] = {32ll << 30, 64ll << 30, 128ll << 30, 256ll << 30};
  o->n.alloc_cpu_milli = cpus[rnd() % 4];
  o->n.alloc_mem = mems[rnd() % 4];
  o->n.alloc_pods = 110;
}

static void make_pod(PodObj* o, int k, const char* node_name) {
  memset(o, 0, sizeof *o);
  ksim_k8s_pod* p = &o->p;
  p->name = S("pod-%d", k);
  p->namespace_ = "default";
  const char* app = S("a%d", (int)(rnd() % NAPP));
  o->label = (ksim_k8s_kv){"app", app};
  p->n_labels = 1;
  p->labels = &o->label;
  p->node_name = node_name;
  static const int64_t cpu[] = {100, 250, 500, 1000, 2000};
  static const int64_t mem[] = {128ll << 20, 256ll << 20, 512ll << 20, 1ll << 30, 2ll << 30};
  if (frand() >= 0.05) {
    o->c.has_cpu = o->c.has_mem = 1;
    o->c.cpu_milli = cpu[rnd() % 5];
    o->c.mem = mem[rnd() % 5];
    o->c.qos_positive = 1;
  }
  if (frand() < 0.2) {
    o->port = (ksim_k8s_port){NULL, "TCP", (int32_t)(8080 + rnd() % 6)};
    o->c.n_ports = 1;
    o->c.ports = &o->port;
  }
  p->n_containers = 1;
  p->containers = &o->c;
  if (frand() < 0.3) {
    o->nsel = (ksim_k8s_kv){"tier", S("%c", "abc"[rnd() % 3])};
    p->n_node_selector = 1;
    p->node_selector = &o->nsel;
  }
  if (frand() < 0.15) {
    o->tol = (ksim_k8s_toleration){"dedicated", "Equal", "gpu", "NoSchedule"};
    p->n_tolerations = 1;
    p->tolerations = &o->tol;
  }
  if (frand() < 0.1) {  /* required anti-affinity against its own app on the node */
    o->anti_ml = (ksim_k8s_kv){"app", app};
    o->anti.selector = (ksim_k8s_label_selector){1, 1, &o->anti_ml, 0, NULL};
    o->anti.topology_key = "kubernetes.io/hostname";
    p->has_pod_anti_affinity = 1;
    p->n_anti_required = 1;
    p->anti_required = &o->anti;
  }
  const double v = frand();
  if (v < 0.12) o->vol = (ksim_k8s_volume){KSIM_K8S_VOL_GCE_PD, frand() < 0.3, S("d%d", (int)(rnd() % 300)), NULL, NULL, 0, NULL};
  else if (v < 0.22) o->vol = (ksim_k8s_volume){KSIM_K8S_VOL_EBS, 0, S("e%d", (int)(rnd() % 300)), NULL, NULL, 0, NULL};
  if (v < 0.22) {
    p->n_volumes = 1;
    p->volumes = &o->vol;
  }
  /* the app's service selects the pod (SelectorFromSet over its selector) */
  o->spread_ml = (ksim_k8s_kv){"app", app};
  o->spread = (ksim_k8s_label_selector){1, 1, &o->spread_ml, 0, NULL};
  o->spread_set = 1;
  if (!node_name) {
    p->n_spread = 1;
    p->spread = &o->spread;
    p->spread_set_selector = &o->spread_set;
  }
}

static ksim_k8s_cluster* snapshot(const NodeObj* nodes, int n, const PodObj* running, int nr, const PodObj* queue, int nq) {
  ksim_k8s_options opt = {10, {0, 0, 0}, -1, -1, 0};
  ksim_k8s_cluster* c = NULL;
  OK(ksim_k8s_create(&opt, &c));
  for (int i = 0; i < n; ++i) OK(ksim_k8s_add_node(c, &nodes[i].n));
  for (int i = 0; i < nr; ++i) OK(ksim_k8s_add_running_pod(c, &running[i].p));
  for (int i = 0; i < nq; ++i) OK(ksim_k8s_add_queued_pod(c, &queue[i].p));
  if (ksim_k8s_build(c)) {
    fprintf(stderr, "build: %s\n", ksim_k8s_last_error(c));
    exit(2);
  }
  return c;
}

int main(int argc, char** argv) {
  const int n = argc > 1 ? atoi(argv[1]) : 200;
  const int nq = argc > 2 ? atoi(argv[2]) : 1500;
  const int nr = n / 2;
  NodeObj* nodes = calloc(n, sizeof *nodes);
  PodObj* running = calloc(nr, sizeof *running);
  PodObj* queue = calloc(nq, sizeof *queue);
  for (int i = 0; i < n; ++i) make_node(&nodes[i], i);
  for (int i = 0; i < nr; ++i) make_pod(&running[i], 100000 + i, nodes[rnd() % n].n.name);
  for (int i = 0; i < nq; ++i) make_pod(&queue[i], i, NULL);

  ksim_config cfg;
  memset(&cfg, 0, sizeof cfg);
  cfg.mode = KSIM_MODE_AUTO;
  cfg.predicates = KSIM_P_CHECK_NODE_CONDITION | KSIM_P_GENERAL | KSIM_P_TAINTS | KSIM_P_MEM_PRESSURE |
                   KSIM_P_DISK_PRESSURE | KSIM_P_INTERPOD_AFFINITY | KSIM_P_DISK_CONFLICT | KSIM_P_MAX_EBS |
                   KSIM_P_MAX_GCE_PD | KSIM_P_MAX_AZURE_DISK | KSIM_P_VOLUME_ZONE;
  cfg.weights[KSIM_W_LEAST_REQUESTED] = 1;
  cfg.weights[KSIM_W_BALANCED] = 1;
  cfg.weights[KSIM_W_TAINT_TOLERATION] = 1;
  cfg.weights[KSIM_W_NODE_AFFINITY] = 1;
  cfg.weights[KSIM_W_INTERPOD_AFFINITY] = 1;
  cfg.weights[KSIM_W_SELECTOR_SPREAD] = 1;
  cfg.collect_reasons = 1;
  cfg.const_score = 10;  /* NodePreferAvoidPods: no owners here */

  /* ---- 1. the queue through ksim_schedule vs the C oracle on the front end's tables ---- */
  ksim_k8s_cluster* A = snapshot(nodes, n, running, nr, queue, nq);
  ksim_handle* h = NULL;
  if (ksim_k8s_open(A, &cfg, 1, &h)) {
    fprintf(stderr, "open: %s\n", ksim_k8s_last_error(A));
    return 2;
  }
  int32_t* got = calloc(nq, 4);
  int32_t* got_r = calloc((size_t)nq * KSIM_NREASONS, 4);
  ksim_stats st;
  OK(ksim_schedule(h, 0, nq, got, got_r, &st));
  uint64_t ctr = 0;
  OK(ksim_get_counter(h, &ctr));

  ksim_node_table nt;
  ksim_class_tables ct;
  ksim_affinity_tables at;
  ksim_volume_tables vt;
  OK(ksim_k8s_tables(A, &nt, &ct, &at, &vt));
  const int64_t N = nt.n_nodes;
  const int32_t S_ = nt.n_scalar, P = nt.port_slots;
  ksim_node_state ns;
  int64_t *rc = malloc(N * 8), *rm = malloc(N * 8), *rg = malloc(N * 8), *re = malloc(N * 8), *zc = malloc(N * 8),
          *zm = malloc(N * 8), *rs = malloc((S_ ? S_ : 1) * N * 8);
  int32_t *pc = malloc(N * 4), *pcount = malloc(N * 4);
  uint64_t* ports = malloc((P ? P : 1) * N * 8);
  memcpy(rc, nt.req_cpu, N * 8); memcpy(rm, nt.req_mem, N * 8); memcpy(rg, nt.req_gpu, N * 8);
  memcpy(re, nt.req_eph, N * 8); memcpy(zc, nt.nz_cpu, N * 8); memcpy(zm, nt.nz_mem, N * 8);
  memcpy(rs, nt.req_scalar, S_ * N * 8); memcpy(pc, nt.pod_count, N * 4); memcpy(pcount, nt.port_count, N * 4);
  memcpy(ports, nt.ports, P * N * 8);
  ns = (ksim_node_state){rc, rm, rg, re, zc, zm, pc, rs, ports, pcount};
  ksim_ref_extra xs;
  memset(&xs, 0, sizeof xs);
  xs.cnt = malloc(at.cnt_len * 4 + 4);
  xs.carried = malloc(at.carried_len * 8 + 8);
  memcpy(xs.cnt, at.cnt, at.cnt_len * 4);
  memcpy(xs.carried, at.carried, at.carried_len * 8);
  xs.vslots = malloc((size_t)vt.vol_slots * N * 8 + 8);
  xs.vcount = malloc(N * 4 + 4);
  memcpy(xs.vslots, vt.slots, (size_t)vt.vol_slots * N * 8);
  memcpy(xs.vcount, vt.slot_count, N * 4);
  const ksim_pod* pods;
  const uint64_t* pp;
  const ksim_scalar_req* ps;
  int64_t npp, nps;
  OK(ksim_k8s_pods(A, &pods, &pp, &npp, &ps, &nps));
  int32_t* want = calloc(nq, 4);
  int32_t* want_r = calloc((size_t)nq * KSIM_NREASONS, 4);
  uint64_t wctr = 0;
  OK(ksim_ref_run_ex(&cfg, &nt, &ns, &ct, at.n_nodes ? &at : NULL, vt.n_nodes ? &vt : NULL, &xs, pods, pp, ps, 0, nq, 1,
                     want, want_r, &wctr));
  int bound = 0;
  for (int k = 0; k < nq; ++k) {
    CHECK(got[k] == want[k], "queue pod %d: device %d, oracle %d", k, got[k], want[k]);
    if (got[k] < 0)
      for (int r = 0; r < KSIM_NREASONS; ++r)
        CHECK(got_r[(size_t)k * KSIM_NREASONS + r] == want_r[(size_t)k * KSIM_NREASONS + r], "pod %d reason %d", k, r);
    bound += got[k] >= 0;
  }
  CHECK(ctr == wctr, "lastNodeIndex %llu vs oracle %llu", (unsigned long long)ctr, (unsigned long long)wctr);
  ksim_destroy(h);

  /* ---- 2. scheduleOne from raw fields: describe → schedule_one(assume) → bind ---- */
  ksim_k8s_cluster* B = snapshot(nodes, n, running, nr, NULL, 0);
  ksim_handle* h2 = NULL;
  if (ksim_k8s_open(B, &cfg, 1, &h2)) {
    fprintf(stderr, "open B: %s\n", ksim_k8s_last_error(B));
    return 2;
  }
  for (int k = 0; k < nq; ++k) {
    ksim_pod d;
    uint64_t kp[8];
    ksim_scalar_req ks[8];
    int32_t nkp = 0, nks = 0;
    int64_t id = -1;
    if (ksim_k8s_describe(B, h2, &queue[k].p, &d, kp, 8, &nkp, ks, 8, &nks, &id)) {
      fprintf(stderr, "describe %d: %s\n", k, ksim_k8s_last_error(B));
      return 2;
    }
    ksim_result res;
    OK(ksim_schedule_one(h2, &d, kp, nkp, ks, nks, KSIM_SCHEDULE_ASSUME, &res));
    CHECK(res.node == got[k], "scheduleOne pod %d: %d, queue run %d", k, res.node, got[k]);
    if (res.node >= 0) OK(ksim_k8s_bind(B, id, res.node));
  }
  uint64_t ctr2 = 0;
  OK(ksim_get_counter(h2, &ctr2));
  CHECK(ctr2 == ctr, "scheduleOne lastNodeIndex %llu vs queue %llu", (unsigned long long)ctr2, (unsigned long long)ctr);
  ksim_destroy(h2);
  ksim_k8s_destroy(A);
  ksim_k8s_destroy(B);
  printf("%s: %d nodes, %d running, %d queued, %d bound, mode %d, lastNodeIndex %llu, %d mismatches\n",
         fails ? "FAIL" : "PASS", n, nr, nq, bound, st.mode, (unsigned long long)ctr, fails);
  return fails ? 1 : 0;
}
