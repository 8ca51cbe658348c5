// ksim_k8s.cpp — the snapshot form of the Kubernetes-field front end (include/ksim_k8s.h): nodes,
// running pods and a queue are added, then interned at once (ksim_k8s_build) into the device tables
// of include/ksim.h, every string comparison the scheduler makes evaluated once per (pod class,
// node label set / taint set).  The semantics (selectors, tolerations, requests, affinity and volume
// identities, table builders) live in ksim_k8s_sem.h, shared with the event-driven scheduler cache
// (ksim_k8s_cache.cpp).  The table layouts and interning rules are the Python host's
// (ksim/ingest.py), which tests/test_k8s_frontend.py compares this with array for array.
#include "ksim_k8s_sem.h"

// ---------------------------------------------------------------- the cluster
struct ksim_k8s_cluster {
  ksim_k8s_options opt{};
  Str err;
  std::vector<NodeObj> nodes_in;
  std::vector<PodObj> running_in, queued_in;
  VolumeIndex vidx_in;  // listers only (PVs, PVCs, storage classes)
  bool built = false;
  // ---- built ----
  std::vector<NodeObj> nodes;  // name-rank order
  std::map<Str, int64_t> index;
  Interns in;
  int32_t port_slots = 0;
  std::vector<int64_t> col_i64[12];  // alloc cpu, mem, gpu, eph, req cpu, mem, gpu, eph, nz cpu, nz mem, (unused)
  std::vector<int32_t> allowed, label_set, taint_set, pod_count, port_count;
  std::vector<uint32_t> flags;
  std::vector<int64_t> alloc_scalar, req_scalar;
  std::vector<uint64_t> ports;
  bool prefer_avoid_nodes = false, node_images = false;
  ClassTab ct;
  // pods
  std::vector<ksim_pod> pods;
  std::vector<uint64_t> pod_ports;
  std::vector<ksim_scalar_req> pod_scalars;
  // affinity
  PolicyArgs pol;  // the open handle's Policy arguments (ksim_k8s_open_policy)
  bool with_affinity = false, spread_active = false;
  AffinityIndex aidx;
  AffTables aff;
  std::vector<int64_t> placed_nodes;     // per running / bound pod: its node
  std::vector<int32_t> placed_ident, placed_aclass;
  // volumes
  bool with_volumes = false;
  VolumeIndex vidx;
  VolSmall vsmall;
  std::vector<uint32_t> vol_zone_ok;
  std::vector<int32_t> vol_slot_count;
  std::vector<uint64_t> vol_slots;
  int32_t vol_S = 0, vol_zone_words = 0;
  bool vol_zone_err = false;
  std::vector<std::map<int32_t, std::array<int32_t, 3>>> mounts;  // per node, key -> rw, ro, pvc
  std::vector<std::vector<int32_t>> mount_order;                  // per node, slot order
  std::set<int32_t> extra_vol_keys;                               // keys of pods described later
  // per-pod drop-in: pods described after the build (their interned ids and volume refs)
  struct Described {
    int32_t ident = -1, aclass = -1;
    std::vector<std::pair<int32_t, uint32_t>> refs;
    PodObj pod;
    int64_t node = -1;  // bound to (ksim_k8s_bind), -1: not placed
  };
  std::vector<Described> described;
  bool dropin = false;        // the affinity tables keep every identity (ksim_k8s_describe)
  ksim_k8s_weights w{};       // the open handle's NodePreferAvoidPods / ImageLocality weights
  bool pa_use_w = false, opened_aff = false, opened_vol = false, opened_zone = false;
  bool opened_svc = false;  // CheckServiceAffinity configured with its Policy arguments
  bool aff_cfg = false, vol_cfg = false;  // the open handle's configuration reads the tables
  int32_t vol_grown_classes = 0;          // volume classes whose zone verdicts the handle holds
  ZoneGroups zone_groups;                 // label sets by zone / region labels (reset with the interns)
};

namespace {

// ---------------------------------------------------------------- build
std::vector<const Labels*> node_labels(const ksim_k8s_cluster* c) {
  std::vector<const Labels*> v;
  for (const NodeObj& x : c->nodes) v.push_back(&x.labels);
  return v;
}

std::vector<Placed> placed_pods(const ksim_k8s_cluster* c) {
  std::vector<Placed> v;
  for (size_t r = 0; r < c->placed_ident.size(); ++r) v.push_back(Placed{c->placed_nodes[r], c->placed_ident[r], c->placed_aclass[r]});
  return v;
}

void build_affinity(ksim_k8s_cluster* c, const std::vector<const PodObj*>& running, const std::vector<const PodObj*>& queued) {
  AffinityIndex& idx = c->aidx;
  idx = AffinityIndex();
  idx.hard_weight = c->opt.hard_weight;
  std::vector<const PodObj*> all(running);
  all.insert(all.end(), queued.begin(), queued.end());
  std::vector<int32_t> idents, aclasses;
  for (const PodObj* p : all) idents.push_back(idx.ident(*p));
  for (size_t k = 0; k < all.size(); ++k) aclasses.push_back(idx.aclass(*all[k], k >= running.size()));
  c->placed_ident.assign(idents.begin(), idents.begin() + running.size());
  c->placed_aclass.assign(aclasses.begin(), aclasses.begin() + running.size());
  build_aff_tables(c->aidx, node_labels(c), placed_pods(c), false, &c->aff);
  for (size_t q = 0; q < queued.size(); ++q) {
    ksim_pod& row = c->pods[q];
    row.aff_ident = c->aff.remap[idents[running.size() + q]];
    row.aff_class = aclasses[running.size() + q] + 1;
  }
}

// One placed pod's mounts on node `node` (NodeInfo.AddPod's volume part).
void add_mounts(ksim_k8s_cluster* c, int64_t node, const std::vector<std::pair<int32_t, uint32_t>>& refs) {
  for (const auto& e : refs) {
    auto ins = c->mounts[node].emplace(e.first, std::array<int32_t, 3>{0, 0, 0});
    if (ins.second) c->mount_order[node].push_back(e.first);
    ins.first->second[(e.second & KSIM_VOL_VIA_PVC) ? 2 : (e.second & KSIM_VOL_READ_ONLY) ? 1 : 0] += 1;
  }
}

void volume_tables(ksim_k8s_cluster* c) {
  VolumeIndex& vi = c->vidx;
  const int64_t n = (int64_t)c->nodes.size();
  const auto& order = c->mount_order;
  vol_small(vi, &c->vsmall);
  std::set<int32_t> qkeys;
  for (const ksim_pod& p : c->pods)
    if (p.vol_class > 0)
      for (const auto& e : vi.class_refs[p.vol_class - 1]) qkeys.insert(e.first);
  for (const auto& e : c->extra_vol_keys) qkeys.insert(e);
  size_t need = 0;
  for (const auto& m : c->mounts) need = std::max(need, m.size());
  need += qkeys.size();
  const int32_t S = c->opt.vol_slots >= 0 ? c->opt.vol_slots : (int32_t)need;
  c->vol_S = S;
  c->vol_slots.assign((size_t)S * n, 0);
  c->vol_slot_count.assign(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    if ((int64_t)order[i].size() > S) fail(KSIM_E_INVAL, "vol_slots too small for running pods");
    for (size_t s = 0; s < order[i].size(); ++s) {
      const int32_t k = order[i][s];
      const auto& m = c->mounts[i][k];
      if (m[0] > 0x7FF || m[1] > 0x7FF || m[2] > 0x3FF)
        fail(KSIM_E_UNSUPPORTED, "more mounts of one volume on a node than a slot counts");
      c->vol_slots[s * n + i] = KSIM_VOL_SLOT(k, m[0], m[1], m[2]);
    }
    c->vol_slot_count[i] = (int32_t)order[i].size();
  }
  // NoVolumeZoneConflict per (class, label set), once per distinct (zone, region) constraint
  c->vol_zone_words = ((int32_t)c->in.label_sets.items.size() + 31) / 32;
  c->vol_zone_ok.clear();
  c->vol_zone_err = false;
  vol_zone_verdicts(vi, c->zone_groups, c->in.label_sets, 0, &c->vol_zone_ok, &c->vol_zone_err);
  if (c->vol_zone_ok.empty()) c->vol_zone_ok.push_back(0);
  c->vol_grown_classes = (int32_t)vi.class_zone.size();
}

void build_volumes(ksim_k8s_cluster* c, const std::vector<const PodObj*>& running) {
  VolumeIndex& vi = c->vidx;
  const int64_t n = (int64_t)c->nodes.size();
  // initial mounts of the running pods
  c->mounts.assign(n, {});
  c->mount_order.assign(n, {});
  for (size_t r = 0; r < running.size(); ++r) {
    std::vector<std::pair<int32_t, uint32_t>> refs;
    std::vector<ZoneEntry> zone;
    bool has_pvc;
    vi.refs(*running[r], false, &refs, &zone, &has_pvc);
    add_mounts(c, c->placed_nodes[r], refs);
  }
  volume_tables(c);
}

void build(ksim_k8s_cluster* c) {
  if (c->built) fail(KSIM_E_STATE, "ksim_k8s_build: already built");
  c->in = Interns();
  c->zone_groups = ZoneGroups();
  c->nodes = c->nodes_in;
  std::stable_sort(c->nodes.begin(), c->nodes.end(), [](const NodeObj& a, const NodeObj& b) { return a.name < b.name; });
  const int64_t n = (int64_t)c->nodes.size();
  for (int64_t i = 0; i < n; ++i) {
    if (!c->index.emplace(c->nodes[i].name, i).second) fail(KSIM_E_INVAL, "duplicate node names");
  }
  for (const NodeObj& x : c->nodes) c->node_images |= x.has_images;
  // ImageLocality's inputs are interned when some node lists images (ingest.Cluster.from_objects)
  c->in.images = c->opt.image_locality > 0 || (c->opt.image_locality == 0 && c->node_images);
  std::vector<const PodObj*> running, queued;
  size_t with_node = 0;
  bool with_pod_affinity = false;
  for (const PodObj& p : c->running_in) {
    with_pod_affinity |= has_pod_affinity(p);
    if (!p.node_name.empty()) ++with_node;
    if (c->index.count(p.node_name)) running.push_back(&p);
  }
  for (const PodObj& p : c->queued_in) {
    with_pod_affinity |= has_pod_affinity(p);
    queued.push_back(&p);
    c->spread_active |= !p.spread.empty();
  }
  c->with_affinity = with_pod_affinity || c->spread_active;
  if (with_pod_affinity && running.size() != with_node)
    fail(KSIM_E_UNSUPPORTED, "running pods bound to nodes outside the snapshot, with inter-pod affinity terms");
  for (const NodeObj& x : c->nodes)
    for (const auto& o : x.other)
      if (is_scalar_resource(o.first)) c->in.scalar_names.get(o.first);
  std::vector<Compiled> compiled;
  for (const PodObj* p : running) compiled.push_back(container_requests(*p));
  for (const PodObj* p : queued) compiled.push_back(container_requests(*p));
  for (const Compiled& cr : compiled) {
    for (const auto& e : cr.pred.scalar) c->in.scalar_names.get(e.first);
    for (const auto& e : cr.add.scalar) c->in.scalar_names.get(e.first);
  }
  if (c->in.scalar_names.items.size() > KSIM_MAX_SCALAR) fail(KSIM_E_UNSUPPORTED, "more than %d scalar resources", KSIM_MAX_SCALAR);
  const int32_t S = (int32_t)c->in.scalar_names.items.size();
  for (auto& v : c->col_i64) v.assign(n, 0);
  c->allowed.assign(n, 0); c->label_set.assign(n, 0); c->taint_set.assign(n, 0); c->pod_count.assign(n, 0);
  c->flags.assign(n, 0);
  c->alloc_scalar.assign((size_t)S * n, 0); c->req_scalar.assign((size_t)S * n, 0);
  for (int64_t i = 0; i < n; ++i) {
    const NodeObj& x = c->nodes[i];
    for (int k = 0; k < 4; ++k) c->col_i64[k][i] = x.alloc[k];
    c->allowed[i] = (int32_t)x.pods;
    for (const auto& o : x.other)
      if (is_scalar_resource(o.first)) c->alloc_scalar[(size_t)c->in.scalar_names.find(o.first) * n + i] += o.second;
    c->flags[i] = node_flags(x);
    c->label_set[i] = c->in.label_set(x);
    c->taint_set[i] = c->in.taint_sets.get(x.taints);
    c->prefer_avoid_nodes |= !x.avoid.empty();
  }
  // running pods: NodeInfo.AddPod
  std::vector<std::vector<uint64_t>> used(n);
  c->placed_nodes.clear();
  for (size_t r = 0; r < running.size(); ++r) {
    const PodObj& p = *running[r];
    const Compiled& cr = compiled[r];
    const int64_t i = c->index[p.node_name];
    c->placed_nodes.push_back(i);
    c->col_i64[4][i] += cr.add.cpu; c->col_i64[5][i] += cr.add.mem; c->col_i64[6][i] += cr.add.gpu; c->col_i64[7][i] += cr.add.eph;
    for (const auto& e : cr.add.scalar) c->req_scalar[(size_t)c->in.scalar_names.find(e.first) * n + i] += e.second;
    c->col_i64[8][i] += cr.nzc; c->col_i64[9][i] += cr.nzm;
    c->pod_count[i] += 1;
    for (const auto& e : host_ports(p)) {
      const uint64_t k = port_key(c->in.ips.get(std::get<0>(e)), c->in.protos.get(std::get<1>(e)), std::get<2>(e));
      if (std::find(used[i].begin(), used[i].end(), k) == used[i].end()) used[i].push_back(k);
    }
  }
  // pod queue
  bool any_vol = false;
  for (const PodObj* p : running) any_vol |= has_pred_volumes(*p);
  for (const PodObj* p : queued) any_vol |= has_pred_volumes(*p);
  c->with_volumes = any_vol;
  if (any_vol) {
    c->vidx = VolumeIndex();
    c->vidx.pvs = c->vidx_in.pvs;
    c->vidx.pvcs = c->vidx_in.pvcs;
    c->vidx.scs = c->vidx_in.scs;
  }
  c->pods.assign(queued.size(), ksim_pod{});
  for (size_t q = 0; q < queued.size(); ++q) {
    encode_pod_row(c->in, c->index, *queued[q], compiled[running.size() + q], &c->pods[q], &c->pod_ports, &c->pod_scalars);
    if (has_pred_volumes(*queued[q])) c->pods[q].vol_class = c->vidx.vclass(*queued[q]);
  }
  if (c->with_affinity) build_affinity(c, running, queued);
  // port slots: enough for everything that could land on one node
  size_t need = 0;
  for (const auto& u : used) need = std::max(need, u.size());
  if (!c->pod_ports.empty()) {
    std::set<uint64_t> distinct(c->pod_ports.begin(), c->pod_ports.end());
    need += distinct.size();
  }
  c->port_slots = c->opt.port_slots >= 0 ? c->opt.port_slots : (int32_t)need;
  const int32_t PS = c->port_slots;
  c->ports.assign((size_t)PS * n, 0);
  c->port_count.assign(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    if ((int64_t)used[i].size() > PS) fail(KSIM_E_INVAL, "port_slots too small for running pods");
    for (size_t s = 0; s < used[i].size(); ++s) c->ports[s * n + i] = used[i][s];
    c->port_count[i] = (int32_t)used[i].size();
  }
  if (c->in.label_sets.items.empty()) c->in.label_sets.get(LabelSetKey{});  // an empty cluster still has tables
  if (c->in.taint_sets.items.empty()) c->in.taint_sets.get({});
  build_class_tab(c->in, &c->ct);
  for (ksim_pod& p : c->pods) p.flags |= c->ct.need[p.cls];
  if (any_vol) build_volumes(c, running);
  c->built = true;
}

int load_volumes(ksim_k8s_cluster* c, ksim_handle* h, bool use_zone) {
  return load_vol_tab(c->vsmall, (int64_t)c->nodes.size(), c->vol_S, c->opt.max_vols, use_zone ? &c->vol_zone_ok : nullptr,
                      c->vol_zone_words, true, c->vol_slots.data(), c->vol_slot_count.data(), h);
}

}  // namespace

// ---------------------------------------------------------------- C-ABI
extern "C" int ksim_k8s_create(const ksim_k8s_options* opt, ksim_k8s_cluster** out) {
  if (!out) return KSIM_E_INVAL;
  auto* c = new ksim_k8s_cluster();
  if (opt) c->opt = *opt;
  else {
    c->opt.hard_weight = 10;
    c->opt.port_slots = -1;
    c->opt.vol_slots = -1;
  }
  default_max_vols(c->opt.max_vols);
  *out = c;
  return KSIM_OK;
}

extern "C" void ksim_k8s_destroy(ksim_k8s_cluster* c) { delete c; }

extern "C" const char* ksim_k8s_last_error(const ksim_k8s_cluster* c) { return c ? c->err.c_str() : "null cluster"; }

extern "C" int ksim_k8s_add_node(ksim_k8s_cluster* c, const ksim_k8s_node* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] {
    if (c->built) fail(KSIM_E_STATE, "ksim_k8s_add_node: the snapshot is built (node events go to ksim_k8s_cache)");
    c->nodes_in.push_back(copy_node(*x));
  });
}

extern "C" int ksim_k8s_add_pv(ksim_k8s_cluster* c, const ksim_k8s_pv* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] { add_pv(&c->vidx_in, *x); });
}

extern "C" int ksim_k8s_add_pvc(ksim_k8s_cluster* c, const ksim_k8s_pvc* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] { add_pvc(&c->vidx_in, *x); });
}

extern "C" int ksim_k8s_add_storage_class(ksim_k8s_cluster* c, const ksim_k8s_storage_class* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] { add_storage_class(&c->vidx_in, *x); });
}

extern "C" int ksim_k8s_add_running_pod(ksim_k8s_cluster* c, const ksim_k8s_pod* p) {
  if (!c || !p) return KSIM_E_INVAL;
  return guard(c, [&] {
    if (c->built) fail(KSIM_E_STATE, "ksim_k8s_add_running_pod: the snapshot is built");
    c->running_in.push_back(copy_pod(*p));
  });
}

extern "C" int ksim_k8s_add_queued_pod(ksim_k8s_cluster* c, const ksim_k8s_pod* p) {
  if (!c || !p) return KSIM_E_INVAL;
  return guard(c, [&] {
    if (c->built) fail(KSIM_E_STATE, "ksim_k8s_add_queued_pod: the snapshot is built");
    c->queued_in.push_back(copy_pod(*p));
  });
}

extern "C" int ksim_k8s_build(ksim_k8s_cluster* c) {
  if (!c) return KSIM_E_INVAL;
  return guard(c, [&] { build(c); });
}

extern "C" int ksim_k8s_open_ex(ksim_k8s_cluster* c, const ksim_config* cfg_in, const ksim_k8s_weights* w_in, ksim_handle** out) {
  return ksim_k8s_open_policy(c, cfg_in, w_in, nullptr, out);
}

extern "C" int ksim_k8s_open_policy(ksim_k8s_cluster* c, const ksim_config* cfg_in, const ksim_k8s_weights* w_in,
                                    const ksim_k8s_policy_args* args, ksim_handle** out) {
  if (!c || !cfg_in || !out) return KSIM_E_INVAL;
  *out = nullptr;
  ksim_handle* h = nullptr;
  const ksim_k8s_weights w = w_in ? *w_in : ksim_k8s_weights{};
  const int rc = guard(c, [&] {
    if (!c->built) fail(KSIM_E_STATE, "ksim_k8s_open: build the snapshot first");
    ksim_config cfg = *cfg_in;
    const uint32_t pr = cfg.predicates;
    PolicyArgs pol;
    if (args) {
      pol.on = true;
      for (int32_t i = 0; i < args->n_presence_labels; ++i) pol.presence_labels.push_back(S(args->presence_labels[i]));
      pol.presence = args->presence != 0;
      for (int32_t i = 0; i < args->n_affinity_labels; ++i) pol.affinity_labels.push_back(S(args->affinity_labels[i]));
      for (int32_t i = 0; i < args->n_label_priorities; ++i) {
        const ksim_k8s_label_priority& q = args->label_priorities[i];
        if (q.weight <= 0) fail(KSIM_E_INVAL, "label priority %s: weight must be positive", S(q.label).c_str());
        pol.label_prios.push_back({S(q.label), {q.presence != 0, q.weight}});
      }
      if (args->n_label_priorities > 0 && cfg.no_priorities)
        fail(KSIM_E_INVAL, "label priorities are prioritizers: cfg.no_priorities must be 0 when n_label_priorities > 0");
      if (args->services_select_pods && ((pr & KSIM_P_SERVICE_AFFINITY) || args->has_service_anti_affinity))
        fail(KSIM_E_UNSUPPORTED, "CheckServiceAffinity / serviceAntiAffinity with services selecting the pods (the Python "
                                 "host builds their service-aware tables)");
    } else if (pr & (KSIM_P_LABEL_PRESENCE | KSIM_P_SERVICE_AFFINITY)) {
      fail(KSIM_E_UNSUPPORTED, "CheckNodeLabelPresence / CheckServiceAffinity need their Policy arguments (ksim_k8s_open_policy)");
    }
    c->pol = pol;
    if (cfg.weights[KSIM_W_NODE_AFFINITY] && !c->ct.bad_classes.empty())
      fail(KSIM_E_UNSUPPORTED, "NodeAffinityPriority: a preferred node-affinity term does not parse");
    if (w.image_locality && c->node_images && !c->in.images)
      fail(KSIM_E_UNSUPPORTED, "ImageLocalityPriority with nodes that list status.images, on a snapshot built without "
                               "image interning (ksim_k8s_options.image_locality = -1)");
    // SelectorSpread's weight stays in its slot even when no queued pod has spread selectors: pods
    // without a spread pair score nothing there (the constant MaxPriority changes no placement), and
    // pods described later (ksim_k8s_describe) may bring selectors
    const uint32_t maxpd = KSIM_P_MAX_EBS | KSIM_P_MAX_GCE_PD | KSIM_P_MAX_AZURE_DISK;
    if (c->with_volumes) {
      if (c->vidx.err_claim && (pr & (maxpd | KSIM_P_VOLUME_ZONE)))
        fail(KSIM_E_UNSUPPORTED, "a PersistentVolumeClaim volume without a claim name (the volume predicates err)");
      if (c->vol_zone_err && (pr & KSIM_P_VOLUME_ZONE))
        fail(KSIM_E_UNSUPPORTED, "NoVolumeZoneConflict with a PVC the PV / PVC listers cannot resolve on a zone-labelled node");
    }
    std::vector<uint8_t> nac;
    std::vector<int32_t> nna;
    std::vector<int64_t> nav, add;
    const bool use_w = cfg.weights[KSIM_W_NODE_AFFINITY] != 0;
    bool pa_on = false;
    const std::vector<int64_t> lab_add = policy_label_add(c->in, pol);
    class_addends(c->ct, w.prefer_avoid, w.image_locality, use_w, &nac, &nna, &nav, &add, &pa_on, &lab_add);
    if (pa_on) cfg.const_score -= 10 * w.prefer_avoid;
    const bool aff = c->with_affinity &&
                     ((pr & KSIM_P_INTERPOD_AFFINITY) ||
                      ((cfg.weights[KSIM_W_INTERPOD_AFFINITY] || cfg.weights[KSIM_W_SELECTOR_SPREAD]) && !cfg.no_priorities));
    const bool vol = c->with_volumes && (pr & (KSIM_P_DISK_CONFLICT | maxpd | KSIM_P_VOLUME_ZONE));
    int e = ksim_create(&cfg, &h);
    if (e) fail(e, "ksim_create: %s", ksim_last_error(nullptr));
    const int64_t n = (int64_t)c->nodes.size();
    ksim_node_table t{};
    t.n_nodes = n;
    t.n_scalar = (int32_t)c->in.scalar_names.items.size();
    t.port_slots = c->port_slots;
    t.alloc_cpu = c->col_i64[0].data(); t.alloc_mem = c->col_i64[1].data(); t.alloc_gpu = c->col_i64[2].data();
    t.alloc_eph = c->col_i64[3].data();
    t.allowed_pods = c->allowed.data(); t.flags = c->flags.data(); t.label_set = c->label_set.data();
    t.taint_set = c->taint_set.data(); t.alloc_scalar = c->alloc_scalar.data();
    t.req_cpu = c->col_i64[4].data(); t.req_mem = c->col_i64[5].data(); t.req_gpu = c->col_i64[6].data();
    t.req_eph = c->col_i64[7].data(); t.nz_cpu = c->col_i64[8].data(); t.nz_mem = c->col_i64[9].data();
    t.pod_count = c->pod_count.data(); t.req_scalar = c->req_scalar.data(); t.ports = c->ports.data();
    t.port_count = c->port_count.data();
    std::vector<uint32_t> flags = c->flags;  // + CheckNodeLabelPresence's verdicts
    if ((pr & KSIM_P_LABEL_PRESENCE) && pol.on) {
      const std::vector<uint8_t> bad = policy_presence_bad(c->in, pol);
      for (int64_t i = 0; i < n; ++i)
        if (bad[c->label_set[i]]) flags[i] |= KSIM_N_LABEL_PRESENCE;
      t.flags = flags.data();
    }
    if ((e = ksim_load_nodes(h, &t))) fail(e, "ksim_load_nodes: %s", ksim_last_error(h));
    std::vector<uint32_t> svc_ok;
    std::vector<uint8_t> svc_need;
    const bool svc = (pr & KSIM_P_SERVICE_AFFINITY) && pol.on;
    if (svc) policy_svc_ok(c->in, c->ct, pol, &svc_ok, &svc_need);
    if ((e = load_class_tab(c->ct, h, w.prefer_avoid, w.image_locality, use_w, svc ? svc_ok.data() : nullptr, &lab_add)))
      fail(e, "ksim_load_classes: %s", ksim_last_error(h));
    if (aff && (e = load_aff_tab(c->aff, n, c->opt.hard_weight, h))) fail(e, "ksim_load_affinity: %s", ksim_last_error(h));
    if (vol && (e = load_volumes(c, h, (pr & KSIM_P_VOLUME_ZONE) != 0))) fail(e, "ksim_load_volumes: %s", ksim_last_error(h));
    c->w = w;
    c->pa_use_w = use_w;
    c->opened_aff = aff;
    c->opened_svc = svc;
    c->opened_vol = vol;
    c->opened_zone = (pr & KSIM_P_VOLUME_ZONE) != 0;
    c->aff_cfg = (pr & KSIM_P_INTERPOD_AFFINITY) ||
                 ((cfg.weights[KSIM_W_INTERPOD_AFFINITY] || cfg.weights[KSIM_W_SELECTOR_SPREAD]) && !cfg.no_priorities);
    c->vol_cfg = (pr & (KSIM_P_DISK_CONFLICT | maxpd | KSIM_P_VOLUME_ZONE)) != 0;
    std::vector<ksim_pod> pods = c->pods;
    for (ksim_pod& p : pods) {
      if (!aff) p.aff_ident = p.aff_class = 0;
      if (!vol) p.vol_class = 0;
      if (svc && svc_need[p.cls]) p.flags |= KSIM_POD_NEED_SVC_AFFINITY;
    }
    if ((e = ksim_load_pods(h, pods.data(), (int64_t)pods.size(), c->pod_ports.data(), (int64_t)c->pod_ports.size(),
                            c->pod_scalars.data(), (int64_t)c->pod_scalars.size())))
      fail(e, "ksim_load_pods: %s", ksim_last_error(h));
  });
  if (rc) {
    if (h) ksim_destroy(h);
    return rc;
  }
  *out = h;
  return KSIM_OK;
}

extern "C" int ksim_k8s_open(ksim_k8s_cluster* c, const ksim_config* cfg, int64_t prefer_avoid_weight, ksim_handle** out) {
  const ksim_k8s_weights w{prefer_avoid_weight, 0};
  return ksim_k8s_open_ex(c, cfg, &w, out);
}

extern "C" int64_t ksim_k8s_node_count(const ksim_k8s_cluster* c) { return c && c->built ? (int64_t)c->nodes.size() : -1; }

extern "C" const char* ksim_k8s_node_name(const ksim_k8s_cluster* c, int64_t rank) {
  if (!c || !c->built || rank < 0 || rank >= (int64_t)c->nodes.size()) return nullptr;
  return c->nodes[rank].name.c_str();
}

extern "C" int64_t ksim_k8s_queue_length(const ksim_k8s_cluster* c) { return c && c->built ? (int64_t)c->pods.size() : -1; }

extern "C" int ksim_k8s_pods(const ksim_k8s_cluster* c, const ksim_pod** pods, const uint64_t** ports, int64_t* n_ports,
                             const ksim_scalar_req** scalars, int64_t* n_scalars) {
  if (!c || !c->built) return KSIM_E_STATE;
  if (pods) *pods = c->pods.data();
  if (ports) *ports = c->pod_ports.data();
  if (n_ports) *n_ports = (int64_t)c->pod_ports.size();
  if (scalars) *scalars = c->pod_scalars.data();
  if (n_scalars) *n_scalars = (int64_t)c->pod_scalars.size();
  return KSIM_OK;
}

extern "C" int ksim_k8s_node_sets(const ksim_k8s_cluster* c, int64_t rank, int32_t* label_set, int32_t* taint_set, uint32_t* flags) {
  if (!c || !c->built || rank < 0 || rank >= (int64_t)c->nodes.size()) return KSIM_E_INVAL;
  if (label_set) *label_set = c->label_set[rank];
  if (taint_set) *taint_set = c->taint_set[rank];
  if (flags) *flags = c->flags[rank];
  return KSIM_OK;
}

extern "C" int64_t ksim_k8s_class_value(const ksim_k8s_cluster* c, int32_t kind, int32_t cls, int32_t set) {
  if (!c || !c->built || cls < 0 || cls >= c->ct.Cn) return -1;
  const ClassTab& t = c->ct;
  switch (kind) {
    case 0: return set < t.L ? (t.sel_ok[(size_t)cls * t.lw + (set >> 5)] >> (set & 31)) & 1u : -1;
    case 1: return set < t.T ? (t.taint_ok[(size_t)cls * t.tw + (set >> 5)] >> (set & 31)) & 1u : -1;
    case 2: return set < t.T ? (t.noexec_ok[(size_t)cls * t.tw + (set >> 5)] >> (set & 31)) & 1u : -1;
    case 3: return set < t.T ? t.tt_val[(size_t)cls * t.val_w + t.tt_class[(size_t)cls * t.T + set]] : -1;
    case 4: return set < t.L ? t.na_w[(size_t)cls * t.L + set] : -1;
    case 5: return set < t.L ? t.im_s[(size_t)cls * t.L + set] : -1;
    default: return -1;
  }
}

extern "C" int ksim_k8s_describe(ksim_k8s_cluster* c, ksim_handle* h, const ksim_k8s_pod* pod, ksim_pod* out,
                                 uint64_t* ports, int32_t port_cap, int32_t* n_ports, ksim_scalar_req* scalars,
                                 int32_t scalar_cap, int32_t* n_scalars, int64_t* pod_id) {
  if (!c || !h || !pod || !out) return KSIM_E_INVAL;
  return guard(c, [&] {
    if (!c->built) fail(KSIM_E_STATE, "ksim_k8s_describe: build and open the snapshot first");
    int64_t hn = -1;
    if (ksim_node_count(h, &hn) != KSIM_OK || hn != (int64_t)c->nodes.size())
      fail(KSIM_E_STATE, "ksim_k8s_describe: the handle has seen node events the snapshot has not (use ksim_k8s_cache)");
    const PodObj p = copy_pod(*pod);
    const Compiled cr = container_requests(p);
    for (const Res* r : {&cr.pred, &cr.add})
      for (const auto& e : r->scalar)
        if (c->in.scalar_names.find(e.first) < 0)
          fail(KSIM_E_UNSUPPORTED, "pod %s: scalar resource %s is not a column of the node table", p.name.c_str(), e.first.c_str());
    const size_t c0 = c->in.classes.items.size();
    ksim_pod row;
    std::vector<uint64_t> pp;
    std::vector<ksim_scalar_req> ps;
    encode_pod_row(c->in, c->index, p, cr, &row, &pp, &ps);
    const int32_t np = row.port_cnt, nsc = row.scalar_cnt;
    if (np > port_cap || nsc > scalar_cap) fail(KSIM_E_INVAL, "pod %s: %d ports / %d scalar requests exceed the arrays", p.name.c_str(), np, nsc);
    for (int32_t k = 0; k < np; ++k) ports[k] = pp[k];
    for (int32_t k = 0; k < nsc; ++k) scalars[k] = ps[k];
    if (n_ports) *n_ports = np;
    if (n_scalars) *n_scalars = nsc;
    int e;
    std::vector<uint32_t> svc_ok;
    std::vector<uint8_t> svc_need;
    const bool svc = c->pol.on && c->opened_svc;
    const bool grew = c->in.classes.items.size() != c0;
    if (grew) build_class_tab(c->in, &c->ct);  // a new pod class: the class tables grow (a superset)
    if (svc) policy_svc_ok(c->in, c->ct, c->pol, &svc_ok, &svc_need);  // once, over the final class table
    if (grew) {
      const std::vector<int64_t> lab_add = policy_label_add(c->in, c->pol);
      if ((e = load_class_tab(c->ct, h, c->w.prefer_avoid, c->w.image_locality, c->pa_use_w, svc ? svc_ok.data() : nullptr,
                              &lab_add)))
        fail(e, "ksim_load_classes: %s", ksim_last_error(h));
    }
    row.flags |= c->ct.need[row.cls];
    if (svc && row.cls < (int32_t)svc_need.size() && svc_need[row.cls]) row.flags |= KSIM_POD_NEED_SVC_AFFINITY;
    ksim_k8s_cluster::Described d;
    // inter-pod affinity / SelectorSpread: identities keep their ids from here on (keep_all)
    const bool takes_part = has_pod_affinity(p) || !p.spread.empty() || c->with_affinity;
    if (c->aff_cfg && takes_part) {
      AffinityIndex& idx = c->aidx;
      if (!c->with_affinity || !c->dropin) {
        if (!c->with_affinity) {  // the snapshot had none: intern its placed pods now
          idx = AffinityIndex();
          idx.hard_weight = c->opt.hard_weight;
          c->placed_ident.clear();
          c->placed_aclass.clear();
          for (const PodObj& r : c->running_in)
            if (c->index.count(r.node_name)) {
              c->placed_ident.push_back(idx.ident(r));
              c->placed_aclass.push_back(idx.aclass(r, false));
            }
          // pods described and bound before any affinity term appeared count as placed pods
          c->placed_nodes.resize(c->placed_ident.size());
          for (auto& x : c->described)
            if (x.node >= 0) {
              x.ident = idx.ident(x.pod);
              x.aclass = idx.aclass(x.pod, true);
              c->placed_nodes.push_back(x.node);
              c->placed_ident.push_back(x.ident);
              c->placed_aclass.push_back(x.aclass);
            }
          c->with_affinity = true;
        }
        c->dropin = true;
      }
      const size_t s0[6] = {idx.keys.items.size(), idx.sels.items.size(), idx.pairs.items.size(), idx.carry.items.size(),
                            idx.idents.items.size(), idx.aclasses.items.size()};
      d.ident = idx.ident(p);
      d.aclass = idx.aclass(p, true);
      const size_t s1[6] = {idx.keys.items.size(), idx.sels.items.size(), idx.pairs.items.size(), idx.carry.items.size(),
                            idx.idents.items.size(), idx.aclasses.items.size()};
      if (!std::equal(s0, s0 + 6, s1) || !c->opened_aff || c->aff.remap.size() != idx.idents.items.size()) {
        build_aff_tables(c->aidx, node_labels(c), placed_pods(c), true, &c->aff);
        if ((e = load_aff_tab(c->aff, (int64_t)c->nodes.size(), c->opt.hard_weight, h))) fail(e, "ksim_load_affinity: %s", ksim_last_error(h));
        c->opened_aff = true;
      }
      row.aff_ident = c->aff.remap[d.ident];
      row.aff_class = d.aclass + 1;
    } else {
      row.aff_ident = row.aff_class = 0;
    }
    // volumes: the first volume pod loads the tables with the bound pods' mounts; later ones grow
    // the small tables in place (ksim_grow_volumes) — the device keeps every node's mounts
    row.vol_class = 0;
    if (c->vol_cfg && has_pred_volumes(p)) {
      if (!c->with_volumes) {
        c->vidx = VolumeIndex();
        c->vidx.pvs = c->vidx_in.pvs;
        c->vidx.pvcs = c->vidx_in.pvcs;
        c->vidx.scs = c->vidx_in.scs;
        std::vector<const PodObj*> running;
        for (const PodObj& r : c->running_in)
          if (c->index.count(r.node_name)) running.push_back(&r);
        build_volumes(c, running);
        c->with_volumes = true;
      }
      VolumeIndex& vi = c->vidx;
      const size_t k0 = vi.keys.items.size(), v0 = vi.class_refs.size();
      const bool claim0 = vi.err_claim;
      row.vol_class = vi.vclass(p);
      if (vi.err_claim && !claim0)
        fail(KSIM_E_UNSUPPORTED, "pod %s: a PersistentVolumeClaim volume without a claim name (the volume predicates err)", p.name.c_str());
      bool has_pvc;
      std::vector<ZoneEntry> zone;
      vi.refs(p, false, &d.refs, &zone, &has_pvc);
      for (const auto& r : d.refs) c->extra_vol_keys.insert(r.first);
      if (!c->opened_vol) {
        volume_tables(c);
        if (c->vol_zone_err && c->opened_zone)
          fail(KSIM_E_UNSUPPORTED, "NoVolumeZoneConflict with a PVC the PV / PVC listers cannot resolve on a zone-labelled node");
        if ((e = load_volumes(c, h, c->opened_zone))) fail(e, "ksim_load_volumes: %s", ksim_last_error(h));
        c->opened_vol = true;
      } else if (vi.keys.items.size() != k0 || vi.class_refs.size() != v0) {
        // a new key or class: the small tables and the new classes' zone verdicts, more slots when
        // a node could now hold more keys than the loaded tables have
        vol_small(vi, &c->vsmall);
        bool zerr = false;
        std::vector<uint32_t> zk;
        vol_zone_verdicts(vi, c->zone_groups, c->in.label_sets, (size_t)c->vol_grown_classes, &zk, &zerr);
        if (c->vol_grown_classes == 0) c->vol_zone_ok.clear();
        c->vol_zone_ok.insert(c->vol_zone_ok.end(), zk.begin(), zk.end());
        if (c->vol_zone_ok.empty()) c->vol_zone_ok.push_back(0);
        c->vol_grown_classes = (int32_t)vi.class_zone.size();
        if (zerr && c->opened_zone)
          fail(KSIM_E_UNSUPPORTED, "NoVolumeZoneConflict with a PVC the PV / PVC listers cannot resolve on a zone-labelled node");
        size_t most = 0;
        for (const auto& m : c->mounts) most = std::max(most, m.size());
        const int32_t want = (int32_t)(most + c->extra_vol_keys.size());
        if (c->opt.vol_slots < 0 && want > c->vol_S) c->vol_S = std::max(want, 2 * c->vol_S);
        if ((e = load_vol_tab(c->vsmall, (int64_t)c->nodes.size(), c->vol_S, c->opt.max_vols,
                              c->opened_zone ? &c->vol_zone_ok : nullptr, c->vol_zone_words, false, nullptr, nullptr, h)))
          fail(e, "ksim_grow_volumes: %s", ksim_last_error(h));
      }
    }
    d.pod = p;
    c->described.push_back(d);
    if (pod_id) *pod_id = (int64_t)c->described.size() - 1;
    *out = row;
  });
}

extern "C" int ksim_k8s_bind(ksim_k8s_cluster* c, int64_t pod_id, int64_t node) {
  if (!c) return KSIM_E_INVAL;
  return guard(c, [&] {
    if (pod_id < 0 || pod_id >= (int64_t)c->described.size()) fail(KSIM_E_INVAL, "ksim_k8s_bind: pod %lld was not described", (long long)pod_id);
    if (node < 0 || node >= (int64_t)c->nodes.size()) fail(KSIM_E_INVAL, "ksim_k8s_bind: node %lld out of range", (long long)node);
    auto& d = c->described[pod_id];
    if (d.node >= 0) fail(KSIM_E_STATE, "ksim_k8s_bind: pod %lld is already bound", (long long)pod_id);
    d.node = node;
    if (c->with_affinity && d.ident >= 0) {
      c->placed_nodes.push_back(node);
      c->placed_ident.push_back(d.ident);
      c->placed_aclass.push_back(d.aclass);
    }
    if (c->with_volumes && !d.refs.empty()) add_mounts(c, node, d.refs);
  });
}

extern "C" int ksim_k8s_tables(ksim_k8s_cluster* c, ksim_node_table* nodes, ksim_class_tables* classes,
                               ksim_affinity_tables* aff, ksim_volume_tables* vol) {
  if (!c || !c->built) return KSIM_E_STATE;
  const int64_t n = (int64_t)c->nodes.size();
  if (nodes) {
    ksim_node_table& t = *nodes;
    t = ksim_node_table{};
    t.n_nodes = n;
    t.n_scalar = (int32_t)c->in.scalar_names.items.size();
    t.port_slots = c->port_slots;
    t.alloc_cpu = c->col_i64[0].data(); t.alloc_mem = c->col_i64[1].data(); t.alloc_gpu = c->col_i64[2].data();
    t.alloc_eph = c->col_i64[3].data();
    t.allowed_pods = c->allowed.data(); t.flags = c->flags.data(); t.label_set = c->label_set.data();
    t.taint_set = c->taint_set.data(); t.alloc_scalar = c->alloc_scalar.data();
    t.req_cpu = c->col_i64[4].data(); t.req_mem = c->col_i64[5].data(); t.req_gpu = c->col_i64[6].data();
    t.req_eph = c->col_i64[7].data(); t.nz_cpu = c->col_i64[8].data(); t.nz_mem = c->col_i64[9].data();
    t.pod_count = c->pod_count.data(); t.req_scalar = c->req_scalar.data(); t.ports = c->ports.data();
    t.port_count = c->port_count.data();
  }
  if (classes) {
    ksim_class_tables& t = *classes;
    const ClassTab& x = c->ct;
    t = ksim_class_tables{};
    t.n_classes = x.Cn; t.n_label_sets = x.L; t.n_taint_sets = x.T;
    t.sel_ok = x.sel_ok.data(); t.taint_ok = x.taint_ok.data(); t.noexec_ok = x.noexec_ok.data();
    t.tt_class = x.tt_class.data(); t.na_class = x.na_class.data(); t.n_tt = x.n_tt.data(); t.n_na = x.n_na.data();
    t.tt_val = x.tt_val.data(); t.na_val = x.na_val.data();
    t.val_width = x.val_w;
  }
  if (aff) {
    *aff = ksim_affinity_tables{};
    if (c->with_affinity) aff_struct(c->aff, n, c->opt.hard_weight, aff);
  }
  if (vol) {
    *vol = ksim_volume_tables{};
    if (c->with_volumes) {
      ksim_volume_tables& t = *vol;
      t.n_keys = (int32_t)c->vsmall.key_filter.size(); t.n_vclass = (int32_t)c->vsmall.vc_filter.size();
      t.n_refs = (int32_t)c->vsmall.refs.size(); t.vol_slots = c->vol_S; t.n_nodes = n;
      for (int k = 0; k < 3; ++k) t.max_vols[k] = c->opt.max_vols[k];
      t.zone_words = c->vol_zone_words;
      t.key_filter = c->vsmall.key_filter.data(); t.vc = c->vsmall.vc.data(); t.vc_filter = c->vsmall.vc_filter.data();
      t.refs = c->vsmall.refs.data(); t.zone_ok = c->vol_zone_ok.data(); t.slots = c->vol_slots.data();
      t.slot_count = c->vol_slot_count.data();
    }
  }
  return KSIM_OK;
}
