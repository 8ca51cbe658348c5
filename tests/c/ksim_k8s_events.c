/*
 * Plain-C scheduleOne loop over the scheduler cache of include/ksim_k8s.h (gcc, the header alone):
 * what a cgo adapter's informer handlers and scheduleOne do — node add / update / remove, pod
 * add / update / remove, assume and forget, Schedule + assume — on a device-resident table, with
 * every scheduling rule in the library.
 *
 * The events come from a script (argv[1]) written by tests/test_c_abi.py from a seeded informer-style
 * stream (tests/events.py); each object is the flattened v1.Node / v1.Pod (the ksim_k8s_* structs, in
 * their field order, as tokens: integers, strings percent-encoded, "-" for "", "~" for NULL, arrays as
 * a count then the elements).  For every SCHEDULE event the program prints one line to argv[2]: the
 * host, "FIT <FitError text>", or "NONODES"; then "COUNTER <lastNodeIndex>".  The test compares the
 * lines with the object oracle's cache (oracle/ksim_ref.py SchedulerCache).  Exit 0 = the loop ran.
 * The summary line also gives the wall time of the ksim_k8s_cache_schedule calls (script parsing
 * excluded): what a cgo adapter's scheduleOne pays per pod (bench.py's per_pod line reads it).
 */
#define _POSIX_C_SOURCE 199309L
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "ksim_k8s.h"

/* ---- arena: everything one event's objects point into ---- */
static char* arena;
static size_t arena_cap, arena_used;
static void* alloc(size_t n) {
  n = (n + 15) & ~(size_t)15;
  if (arena_used + n > arena_cap) {
    fprintf(stderr, "arena exhausted\n");
    exit(2);
  }
  void* p = arena + arena_used;
  arena_used += n;
  memset(p, 0, n);
  return p;
}

/* ---- tokens ---- */
static FILE* in;
static char tok[1 << 16];
static int next_token(void) {
  int c;
  while ((c = fgetc(in)) == ' ' || c == '\n' || c == '\t' || c == '\r') {
  }
  if (c == EOF) return 0;
  size_t n = 0;
  while (c != EOF && c != ' ' && c != '\n' && c != '\t' && c != '\r') {
    if (n + 1 < sizeof tok) tok[n++] = (char)c;
    c = fgetc(in);
  }
  tok[n] = 0;
  return 1;
}
static void need(void) {
  if (!next_token()) {
    fprintf(stderr, "unexpected end of script\n");
    exit(2);
  }
}
static int64_t rd_i(void) {
  need();
  return strtoll(tok, NULL, 10);
}
static int hexv(char c) { return c >= '0' && c <= '9' ? c - '0' : c >= 'a' && c <= 'f' ? c - 'a' + 10 : c - 'A' + 10; }
static const char* rd_s(void) {
  need();
  if (!strcmp(tok, "~")) return NULL;
  if (!strcmp(tok, "-")) return "";
  char* out = (char*)alloc(strlen(tok) + 1);
  size_t k = 0;
  for (const char* p = tok; *p; ++p) {
    if (*p == '%' && p[1] && p[2]) {
      out[k++] = (char)(hexv(p[1]) * 16 + hexv(p[2]));
      p += 2;
    } else {
      out[k++] = *p;
    }
  }
  out[k] = 0;
  return out;
}
#define RD_ARR(T, n, ptr, fn)                                  \
  do {                                                         \
    n = (int32_t)rd_i();                                       \
    T* a_ = (T*)alloc(sizeof(T) * (size_t)(n > 0 ? n : 1));   \
    for (int32_t i_ = 0; i_ < n; ++i_) fn(&a_[i_]);            \
    ptr = a_;                                                  \
  } while (0)

static void rd_str(const char** p) { *p = rd_s(); }
static void rd_i32(int32_t* p) { *p = (int32_t)rd_i(); }
static void rd_kv(ksim_k8s_kv* x) { x->key = rd_s(); x->value = rd_s(); }
static void rd_req(ksim_k8s_req* x) {
  x->key = rd_s();
  x->op = rd_s();
  const char** v;
  RD_ARR(const char*, x->n_values, v, rd_str);
  x->values = v;
}
static void rd_node_term(ksim_k8s_node_term* x) { RD_ARR(ksim_k8s_req, x->n_reqs, x->reqs, rd_req); }
static void rd_pref_term(ksim_k8s_pref_node_term* x) {
  x->weight = (int32_t)rd_i();
  rd_node_term(&x->preference);
}
static void rd_label_selector(ksim_k8s_label_selector* x) {
  x->present = (int32_t)rd_i();
  RD_ARR(ksim_k8s_kv, x->n_match_labels, x->match_labels, rd_kv);
  RD_ARR(ksim_k8s_req, x->n_exprs, x->exprs, rd_req);
}
static void rd_pod_term(ksim_k8s_pod_term* x) {
  rd_label_selector(&x->selector);
  const char** v;
  RD_ARR(const char*, x->n_namespaces, v, rd_str);
  x->namespaces = v;
  x->topology_key = rd_s();
  x->weight = (int32_t)rd_i();
}
static void rd_taint(ksim_k8s_taint* x) { x->key = rd_s(); x->value = rd_s(); x->effect = rd_s(); }
static void rd_toleration(ksim_k8s_toleration* x) { x->key = rd_s(); x->op = rd_s(); x->value = rd_s(); x->effect = rd_s(); }
static void rd_resource(ksim_k8s_resource* x) { x->name = rd_s(); x->value = rd_i(); }
static void rd_port(ksim_k8s_port* x) { x->host_ip = rd_s(); x->protocol = rd_s(); x->host_port = (int32_t)rd_i(); }
static void rd_container(ksim_k8s_container* x) {
  x->has_cpu = (int32_t)rd_i(); x->has_mem = (int32_t)rd_i();
  x->cpu_milli = rd_i(); x->mem = rd_i(); x->gpu = rd_i(); x->eph = rd_i();
  RD_ARR(ksim_k8s_resource, x->n_other, x->other, rd_resource);
  x->qos_positive = (int32_t)rd_i();
  RD_ARR(ksim_k8s_port, x->n_ports, x->ports, rd_port);
  x->image = rd_s();
}
static void rd_volume(ksim_k8s_volume* x) {
  x->kind = (int32_t)rd_i(); x->read_only = (int32_t)rd_i();
  x->id = rd_s(); x->pool = rd_s(); x->image = rd_s();
  const char** v;
  RD_ARR(const char*, x->n_monitors, v, rd_str);
  x->monitors = v;
}
static void rd_pod(ksim_k8s_pod* x) {
  x->name = rd_s(); x->namespace_ = rd_s();
  RD_ARR(ksim_k8s_kv, x->n_labels, x->labels, rd_kv);
  x->deleting = (int32_t)rd_i();
  x->node_name = rd_s();
  RD_ARR(ksim_k8s_container, x->n_containers, x->containers, rd_container);
  RD_ARR(ksim_k8s_container, x->n_init_containers, x->init_containers, rd_container);
  RD_ARR(ksim_k8s_kv, x->n_node_selector, x->node_selector, rd_kv);
  x->has_node_affinity = (int32_t)rd_i(); x->has_required = (int32_t)rd_i();
  RD_ARR(ksim_k8s_node_term, x->n_required_terms, x->required_terms, rd_node_term);
  RD_ARR(ksim_k8s_pref_node_term, x->n_preferred, x->preferred, rd_pref_term);
  RD_ARR(ksim_k8s_toleration, x->n_tolerations, x->tolerations, rd_toleration);
  x->has_pod_affinity = (int32_t)rd_i(); x->has_pod_anti_affinity = (int32_t)rd_i();
  RD_ARR(ksim_k8s_pod_term, x->n_affinity_required, x->affinity_required, rd_pod_term);
  RD_ARR(ksim_k8s_pod_term, x->n_affinity_preferred, x->affinity_preferred, rd_pod_term);
  RD_ARR(ksim_k8s_pod_term, x->n_anti_required, x->anti_required, rd_pod_term);
  RD_ARR(ksim_k8s_pod_term, x->n_anti_preferred, x->anti_preferred, rd_pod_term);
  RD_ARR(ksim_k8s_volume, x->n_volumes, x->volumes, rd_volume);
  RD_ARR(ksim_k8s_label_selector, x->n_spread, x->spread, rd_label_selector);
  int32_t n_set;
  int32_t* set;
  RD_ARR(int32_t, n_set, set, rd_i32);
  x->spread_set_selector = set;
  x->avoid_ctrl_kind = rd_s(); x->avoid_ctrl_uid = rd_s();
  x->uid = rd_s();
}
static void rd_condition(ksim_k8s_condition* x) { x->type = rd_s(); x->status = rd_s(); }
static void rd_avoid(ksim_k8s_avoid* x) { x->has_controller = (int32_t)rd_i(); x->kind = rd_s(); x->uid = rd_s(); }
static void rd_image(ksim_k8s_image* x) {
  const char** v;
  RD_ARR(const char*, x->n_names, v, rd_str);
  x->names = v;
  x->size_bytes = rd_i();
}
static void rd_node(ksim_k8s_node* x) {
  x->name = rd_s();
  RD_ARR(ksim_k8s_kv, x->n_labels, x->labels, rd_kv);
  RD_ARR(ksim_k8s_taint, x->n_taints, x->taints, rd_taint);
  x->unschedulable = (int32_t)rd_i();
  RD_ARR(ksim_k8s_condition, x->n_conditions, x->conditions, rd_condition);
  x->alloc_cpu_milli = rd_i(); x->alloc_mem = rd_i(); x->alloc_gpu = rd_i(); x->alloc_eph = rd_i(); x->alloc_pods = rd_i();
  RD_ARR(ksim_k8s_resource, x->n_alloc_other, x->alloc_other, rd_resource);
  RD_ARR(ksim_k8s_avoid, x->n_avoid, x->avoid, rd_avoid);
  x->has_images = (int32_t)rd_i();
  RD_ARR(ksim_k8s_image, x->n_images, x->images, rd_image);
}

static int cmp_d(const void* a, const void* b) {
  const double x = *(const double*)a, y = *(const double*)b;
  return x < y ? -1 : x > y;
}

int main(int argc, char** argv) {
  if (argc < 3) {
    fprintf(stderr, "usage: %s <script> <out>\n", argv[0]);
    return 2;
  }
  in = fopen(argv[1], "r");
  FILE* out = fopen(argv[2], "w");
  if (!in || !out) {
    perror("open");
    return 2;
  }
  arena_cap = 64u << 20;
  arena = (char*)malloc(arena_cap);
  /* header: the scheduler's configuration (ksim_k8s_cache_options) */
  ksim_k8s_cache_options opt;
  memset(&opt, 0, sizeof opt);
  need();
  if (strcmp(tok, "CONFIG")) return 2;
  opt.cfg.device = (int32_t)rd_i();
  opt.cfg.mode = (int32_t)rd_i();
  opt.cfg.predicates = (uint32_t)rd_i();
  for (int k = 0; k < KSIM_NW; ++k) opt.cfg.weights[k] = rd_i();
  opt.cfg.no_priorities = (int32_t)rd_i();
  opt.cfg.collect_reasons = 1;
  opt.cfg.const_score = rd_i();
  opt.extra.prefer_avoid = rd_i();
  opt.extra.image_locality = rd_i();
  opt.hard_weight = (int32_t)rd_i();
  opt.check_volume_binding = (int32_t)rd_i();
  ksim_k8s_cache* c = NULL;
  if (ksim_k8s_cache_create(&opt, &c)) {
    fprintf(stderr, "ksim_k8s_cache_create: %s\n", ksim_k8s_cache_last_error(NULL));
    return 1;
  }
  int64_t events = 0, decisions = 0, fits = 0;
  double* lat = (double*)malloc(sizeof(double) * (1 << 22));
  int64_t nlat = 0;
  char msg[4096];
  while (next_token()) {
    arena_used = 0;
    char verb[32];
    strncpy(verb, tok, sizeof verb - 1);
    verb[sizeof verb - 1] = 0;
    ksim_k8s_node n1, n2;
    ksim_k8s_pod p1, p2;
    memset(&n1, 0, sizeof n1); memset(&n2, 0, sizeof n2); memset(&p1, 0, sizeof p1); memset(&p2, 0, sizeof p2);
    int rc = 0;
    ++events;
    if (!strcmp(verb, "ADD_NODE")) {
      rd_node(&n1);
      rc = ksim_k8s_cache_add_node(c, &n1);
    } else if (!strcmp(verb, "UPDATE_NODE")) {
      rd_node(&n1);
      rd_node(&n2);
      rc = ksim_k8s_cache_update_node(c, &n1, &n2);
    } else if (!strcmp(verb, "REMOVE_NODE")) {
      rd_node(&n1);
      rc = ksim_k8s_cache_remove_node(c, &n1);
    } else if (!strcmp(verb, "ADD_POD")) {
      rd_pod(&p1);
      rc = ksim_k8s_cache_add_pod(c, &p1);
    } else if (!strcmp(verb, "UPDATE_POD")) {
      rd_pod(&p1);
      rd_pod(&p2);
      rc = ksim_k8s_cache_update_pod(c, &p1, &p2);
    } else if (!strcmp(verb, "REMOVE_POD")) {
      rd_pod(&p1);
      rc = ksim_k8s_cache_remove_pod(c, &p1);
    } else if (!strcmp(verb, "FORGET_POD")) {
      rd_pod(&p1);
      rc = ksim_k8s_cache_forget_pod(c, &p1);
    } else if (!strcmp(verb, "SCHEDULE")) {
      rd_pod(&p1);
      ksim_result res;
      struct timespec t0, t1;
      clock_gettime(CLOCK_MONOTONIC, &t0);
      rc = ksim_k8s_cache_schedule(c, &p1, KSIM_SCHEDULE_ASSUME, &res);
      clock_gettime(CLOCK_MONOTONIC, &t1);
      if (nlat < (1 << 22)) lat[nlat++] = (double)(t1.tv_sec - t0.tv_sec) * 1e6 + (double)(t1.tv_nsec - t0.tv_nsec) * 1e-3;
      ++decisions;
      if (rc == KSIM_E_NO_NODES) {
        fprintf(out, "NONODES\n");
        rc = 0;
      } else if (rc == 0 && res.node < 0) {
        ksim_k8s_cache_fit_error(c, &res, msg, sizeof msg);
        fprintf(out, "FIT %s\n", msg);
        ++fits;
      } else if (rc == 0) {
        fprintf(out, "%s\n", ksim_k8s_cache_node_name(c, res.node));
      }
    } else {
      fprintf(stderr, "unknown event %s\n", verb);
      return 2;
    }
    if (rc) {
      fprintf(stderr, "event %lld (%s): %d %s\n", (long long)events, verb, rc, ksim_k8s_cache_last_error(c));
      return 1;
    }
  }
  uint64_t ctr = 0;
  if (ksim_get_counter(ksim_k8s_cache_handle(c), &ctr)) return 1;
  fprintf(out, "COUNTER %llu\n", (unsigned long long)ctr);
  fclose(out);
  double sum = 0;
  for (int64_t i = 0; i < nlat; ++i) sum += lat[i];
  qsort(lat, (size_t)nlat, sizeof(double), cmp_d);
  printf("ksim_k8s_events: %lld events, %lld decisions (%lld FitErrors), %lld nodes listed; schedule calls: mean %.2f us, "
         "p50 %.2f us, p90 %.2f us, p99 %.2f us\n",
         (long long)events, (long long)decisions, (long long)fits, (long long)ksim_k8s_cache_node_count(c),
         nlat ? sum / (double)nlat : 0.0, nlat ? lat[nlat / 2] : 0.0, nlat ? lat[nlat * 9 / 10] : 0.0,
         nlat ? lat[nlat * 99 / 100] : 0.0);
  free(lat);
  ksim_k8s_cache_destroy(c);
  free(arena);
  return 0;
}
