// ksim_k8s_cache.cpp — the event-driven scheduler cache of the Kubernetes-field front end
// (include/ksim_k8s.h, "The scheduler cache"): schedulercache.Cache (schedulercache/cache.go:125-393)
// and genericScheduler.Schedule (core/generic_scheduler.go:112-198) over the device-resident node
// table, fed by the informer events the reference's config factory wires (factory/factory.go:596,
// 613, 695, 740, 755, 841) and by scheduleOne's assume / forget (scheduler.go:366-412).  It is the
// C++ restatement of ksim/cache.py's SchedulerCache (same bookkeeping, same refusals), so a cgo
// adapter can mirror the reference's cache without re-porting any rule:
//  - nodes: SetNode's static columns from the node object (labels / taints / images / preferAvoidPods
//    interned into label and taint sets, the class tables grown when a set is new), the dynamic
//    columns of the pods its NodeInfo already holds, inserted at its bytewise name rank;
//  - pods: NodeInfo.AddPod / RemovePod on the device (ksim_pod_add / _remove) for listed nodes; the
//    host keeps pod identity, the encodings and the pods of unlisted nodes;
//  - inter-pod affinity / SelectorSpread: an index kept across calls (predicates/metadata.go:127-190),
//    tables reloaded only when it grows by something the device must hold or after a node event;
//  - volumes: the device keeps every node's mounts; new keys / classes grow the small tables
//    (ksim_grow_volumes), a node event reloads them with the host's mount view.
#include <chrono>
#include <cstdio>
#include <memory>

#include "ksim_k8s_sem.h"

namespace {

struct Enc {  // a pod's descriptor and the arrays its offsets index
  ksim_pod row{};
  std::vector<uint64_t> ports;
  std::vector<ksim_scalar_req> scalars;
};

struct PodRec {
  PodObj pod;
  Enc enc;
};

struct Info {  // one cache.nodes entry (NodeInfo)
  bool has_node = false;  // AddNode seen and no RemoveNode since
  NodeObj node;
  Str mem, disk;          // SetNode's last MemoryPressure / DiskPressure status ("" none)
  std::map<Str, PodRec> pods;
};

// getPodKey (schedulercache/node_info.go:497-503): the UID; pods without one by namespace/name.
Str pod_key(const PodObj& p) { return !p.uid.empty() ? p.uid : p.ns + "/" + p.name; }

constexpr uint32_t MAXPD_BITS = KSIM_P_MAX_EBS | KSIM_P_MAX_GCE_PD | KSIM_P_MAX_AZURE_DISK;
constexpr uint32_t VOLUME_BITS = KSIM_P_DISK_CONFLICT | MAXPD_BITS | KSIM_P_VOLUME_ZONE;

}  // namespace

struct ksim_k8s_cache {
  Str err;
  ksim_k8s_cache_options opt{};
  ksim_handle* h = nullptr;
  Interns in;
  ClassTab ct;
  std::array<size_t, 3> tables_for{{SIZE_MAX, SIZE_MAX, SIZE_MAX}};  // (L, T, classes) of the loaded class tables
  bool need_na = false, aff_wanted = false, vol_on = false, use_zone = false;
  PolicyArgs pol;                    // a Policy's arguments (ksim_k8s_cache_options.policy, copied)
  bool pol_presence = false, pol_svc = false;
  std::vector<uint32_t> svc_ok;      // CheckServiceAffinity's (class, label set) table
  std::vector<uint8_t> svc_need;
  std::vector<Str> names;            // listed nodes, ascending bytewise (= name rank)
  std::map<Str, int64_t> rank;
  bool rank_valid = true;
  std::map<Str, Info> infos;         // cache.nodes
  std::map<Str, PodObj> pod_states;  // cache.podStates: key -> pod
  std::set<Str> assumed;             // cache.assumedPods
  // inter-pod affinity / SelectorSpread
  bool aff_on = false;               // some scheduled or cached pod had terms or spread selectors
  std::unique_ptr<AffinityIndex> aidx;
  bool have_sig = false;
  std::array<size_t, 6> aff_sig{};   // index sizes at the last load (sels, pairs, carry, keys, aclasses, idents)
  std::vector<int32_t> aff_remap;    // identity -> aff_ident of the loaded tables
  bool aff_check = false;            // an affinity pod may be cached on an unlisted node: rebuild next time
  // volumes
  VolumeIndex vidx;
  bool vol_loaded = false, vol_dirty = false;
  std::array<size_t, 3> vol_key{};   // (keys, classes, label sets) the loaded tables cover
  std::map<Str, std::map<int32_t, std::array<int32_t, 3>>> vol_mounts;  // node -> key -> rw, ro, pvc
  size_t vol_max = 0;                // an upper bound of the keys mounted on any node
  int32_t vol_S = 0;
  std::vector<uint32_t> vol_zone;    // NoVolumeZoneConflict verdicts [class][words]
  size_t vol_zone_classes = 0;
  int32_t vol_zone_words = 0;
  bool vol_zone_err = false;
  int64_t stats[4] = {0, 0, 0, 0};   // affinity loads, volume loads, volume grows, class loads
  // KSIM_CACHE_PROFILE=1 (diagnostic): ns per Schedule phase — encode, volume errors, volume sync,
  // affinity sync, ksim_schedule_one, bookkeeping; [6] calls — printed by ksim_k8s_cache_destroy
  int64_t prof[7] = {0, 0, 0, 0, 0, 0, 0};
  int64_t prof_seen = 0;              // Schedule calls so far (KSIM_CACHE_PROFILE_SKIP: untimed head)
  size_t zoned_upto = 0;              // label sets scanned for zone / region labels
  ZoneGroups zone_groups;             // label sets by their zone / region labels (volume zone verdicts)
  bool zoned = false;
  VolSmall vs;                        // the small volume tables as last loaded (grows append to them)
};

namespace {

using Cache = ksim_k8s_cache;

void check(Cache* c, int rc, const char* what) {
  if (rc) fail(rc, "%s: %s", what, ksim_last_error(c->h));
}

const std::map<Str, int64_t>& ranks(Cache* c) {
  if (!c->rank_valid) {
    c->rank.clear();
    for (size_t i = 0; i < c->names.size(); ++i) c->rank.emplace(c->names[i], (int64_t)i);
    c->rank_valid = true;
  }
  return c->rank;
}

int64_t rank_of(Cache* c, const Str& name) {
  const auto& r = ranks(c);
  auto it = r.find(name);
  return it == r.end() ? -1 : it->second;
}

// The class tables, reloaded when a label set, taint set or pod class was interned since.
void load_tables(Cache* c) {
  const std::array<size_t, 3> key{{c->in.label_sets.items.size(), c->in.taint_sets.items.size(), c->in.classes.items.size()}};
  if (key == c->tables_for) return;
  build_class_tab(c->in, &c->ct);
  const std::vector<int64_t> lab_add = policy_label_add(c->in, c->pol);  // a Policy's label priorities
  if (c->pol_svc) policy_svc_ok(c->in, c->ct, c->pol, &c->svc_ok, &c->svc_need);
  check(c, load_class_tab(c->ct, c->h, c->opt.extra.prefer_avoid, c->opt.extra.image_locality, c->need_na,
                          c->pol_svc ? c->svc_ok.data() : nullptr, &lab_add), "ksim_load_classes");
  c->tables_for = key;
  c->stats[3] += 1;
}

int32_t scalar_id(Cache* c, const Str& name) {
  if (c->in.scalar_names.find(name) < 0 && c->in.scalar_names.items.size() >= KSIM_MAX_SCALAR)
    fail(KSIM_E_UNSUPPORTED, "more than %d scalar resources", KSIM_MAX_SCALAR);
  return c->in.scalar_names.get(name);
}

// A pod's descriptor (SchedulerCache._encode): its class interned (the class tables grown), the
// class's KSIM_POD_NEED_* flags, its volume class when a volume predicate is configured.
Enc encode(Cache* c, const PodObj& p) {
  const Compiled cr = container_requests(p);
  for (const Res* r : {&cr.pred, &cr.add})
    for (const auto& e : r->scalar) scalar_id(c, e.first);
  Enc e;
  encode_pod_row(c->in, ranks(c), p, cr, &e.row, &e.ports, &e.scalars);
  load_tables(c);
  const int32_t cls = e.row.cls;
  if (c->need_na && c->ct.bad_classes.count(cls))
    fail(KSIM_E_UNSUPPORTED, "NodeAffinityPriority: a preferred node-affinity term does not parse");
  e.row.flags |= c->ct.need[cls];
  if (c->pol_svc && cls < (int32_t)c->svc_need.size() && c->svc_need[cls]) e.row.flags |= KSIM_POD_NEED_SVC_AFFINITY;
  if (c->vol_on && has_pred_volumes(p)) e.row.vol_class = c->vidx.vclass(p);
  return e;
}

// ---------------------------------------------------------------- volumes
void mount(Cache* c, const Str& name, const Enc& e, int sign) {
  const int32_t vc = e.row.vol_class;
  if (!vc || !c->vol_on) return;
  auto& m = c->vol_mounts[name];
  for (const auto& r : c->vidx.class_refs[vc - 1]) {
    auto& x = m[r.first];
    x[(r.second & KSIM_VOL_VIA_PVC) ? 2 : (r.second & KSIM_VOL_READ_ONLY) ? 1 : 0] += sign;
    if (!x[0] && !x[1] && !x[2]) m.erase(r.first);
  }
  c->vol_max = std::max(c->vol_max, m.size());
}

// SchedulerCache._sync_volumes: the device's volume tables current for a call — first load (when a
// volume pod needs them) and after every node event: the full tables with the host's mounts;
// otherwise, when new keys / classes appeared or a node could hold more keys than loaded:
// ksim_grow_volumes with the small tables only (the device keeps every node's mounts).
void sync_volumes(Cache* c, bool need, const Enc* e) {
  if (!c->vol_on) return;
  VolumeIndex& vi = c->vidx;
  const std::array<size_t, 3> key{{vi.key_filter.size(), vi.class_refs.size(), c->in.label_sets.items.size()}};
  const int32_t vc = e ? e->row.vol_class : 0;
  const size_t want = c->vol_max + (vc ? vi.class_refs[vc - 1].size() : 0);
  if (!c->vol_dirty && !c->vol_loaded && !need) return;
  if (!c->vol_dirty && c->vol_loaded) {
    if (c->vol_key == key && (int64_t)want <= c->vol_S) return;
    if (c->vol_key[2] == key[2]) {
      if (key[1] > c->vol_zone_classes) {
        vol_zone_verdicts(vi, c->zone_groups, c->in.label_sets, c->vol_zone_classes, &c->vol_zone, &c->vol_zone_err);
        c->vol_zone_classes = key[1];
      }
      const int32_t S = std::max<int32_t>(c->vol_S, (int32_t)(2 * want));
      vol_small_append(vi, &c->vs);
      check(c, load_vol_tab(c->vs, (int64_t)c->names.size(), S, c->opt.max_vols, c->use_zone ? &c->vol_zone : nullptr,
                            c->vol_zone_words, false, nullptr, nullptr, c->h),
            "ksim_grow_volumes");
      c->vol_key = key;
      c->vol_S = S;
      c->stats[2] += 1;
      return;
    }
  }
  const int64_t n = (int64_t)c->names.size();
  c->vol_zone.clear();
  c->vol_zone_err = false;
  vol_zone_verdicts(vi, c->zone_groups, c->in.label_sets, 0, &c->vol_zone, &c->vol_zone_err);
  c->vol_zone_classes = key[1];
  c->vol_zone_words = ((int32_t)key[2] + 31) / 32;
  const int32_t S = std::max<int32_t>((int32_t)(2 * want), 8);
  std::vector<uint64_t> slots((size_t)S * n, 0);
  std::vector<int32_t> count(n, 0);
  for (int64_t i = 0; i < n; ++i) {
    auto it = c->vol_mounts.find(c->names[i]);
    if (it == c->vol_mounts.end()) continue;
    int32_t s = 0;
    for (const auto& m : it->second) {
      const auto& x = m.second;
      if (x[0] > 0x7FF || x[1] > 0x7FF || x[2] > 0x3FF) fail(KSIM_E_UNSUPPORTED, "more mounts of one volume on a node than a slot counts");
      slots[(size_t)s * n + i] = KSIM_VOL_SLOT(m.first, x[0], x[1], x[2]);
      ++s;
    }
    count[i] = s;
  }
  vol_small(vi, &c->vs);
  check(c, load_vol_tab(c->vs, n, S, c->opt.max_vols, c->use_zone ? &c->vol_zone : nullptr, c->vol_zone_words, true,
                        slots.data(), count.data(), c->h),
        "ksim_load_volumes");
  c->vol_key = key;
  c->vol_S = S;
  c->vol_dirty = false;
  c->vol_loaded = true;
  c->stats[1] += 1;
}

// The error paths a pod to be scheduled would take (VolumeIndex.pod_errors) → refusals for the
// configured keys (SchedulerCache._check_volume_errors): the reference's findNodesThatFit would
// return the predicate's error and scheduleOne would requeue the pod.
void check_volume_errors(Cache* c, const PodObj& p) {
  VolumeIndex& vi = c->vidx;
  // some label set carries a zone / region label (label sets are only ever added: scan the new ones)
  for (; c->zoned_upto < c->in.label_sets.items.size(); ++c->zoned_upto) {
    const Labels& l = c->in.label_sets.items[c->zoned_upto].labels;
    c->zoned |= l.count(ZONE_LABEL) || l.count(REGION_LABEL);
  }
  const bool zoned = c->zoned;
  bool claim = false, zone = false, binding = false;
  for (const Volume& v : p.vols) {
    if (v.kind != KSIM_K8S_VOL_PVC) continue;
    if (v.id.empty()) {
      claim = true;
      continue;
    }
    if (zoned && vi.zone_entry(p.ns, v.id).kind == 1) zone = true;
    auto pc = vi.pvcs.find({p.ns, v.id});
    const PV* pv = nullptr;
    if (pc != vi.pvcs.end()) {
      auto it = vi.pvs.find(pc->second.volume_name);
      if (it != vi.pvs.end()) pv = &it->second;
    }
    if (!pv || pv->node_affinity) binding = true;
  }
  const uint32_t pr = c->opt.cfg.predicates;
  if (claim && (pr & (MAXPD_BITS | KSIM_P_VOLUME_ZONE)))
    fail(KSIM_E_UNSUPPORTED, "a PersistentVolumeClaim volume without a claim name (the volume predicates err)");
  if (binding && c->opt.check_volume_binding)
    fail(KSIM_E_UNSUPPORTED, "CheckVolumeBinding with a PVC that is not bound to a PV without node affinity");
  if (zone && (pr & KSIM_P_VOLUME_ZONE))
    fail(KSIM_E_UNSUPPORTED, "NoVolumeZoneConflict with a PVC the listers cannot resolve on a zone-labelled cluster");
}

// ---------------------------------------------------------------- inter-pod affinity / SelectorSpread
std::array<size_t, 6> aff_signature(const AffinityIndex& idx) {
  return {{idx.sels.items.size(), idx.pairs.items.size(), idx.carry.items.size(), idx.keys.items.size(),
           idx.aclasses.items.size(), idx.idents.items.size()}};
}

// Nothing the device tables hold changed since the last load, except new identities that no
// selector matches (their aff_ident is 0: they count toward nothing).
bool grew_only_dead(const Cache* c, const AffinityIndex& idx) {
  const auto sig = aff_signature(idx);
  for (int k = 0; k < 5; ++k)
    if (sig[k] != c->aff_sig[k]) return false;
  for (size_t i = c->aff_sig[5]; i < idx.idents.items.size(); ++i)
    for (const SelItem& s : idx.sels.items)
      if (AffinityIndex::sel_matches(idx.idents.items[i], s)) return false;
  return true;
}

// The tables over the pods cached on listed nodes (counts from the host's view), loaded.
void aff_rebuild(Cache* c, AffinityIndex& idx) {
  std::vector<Placed> placed;
  for (auto& kv : c->infos) {
    const int64_t r = rank_of(c, kv.first);
    for (auto& pr : kv.second.pods) {
      const PodObj& p = pr.second.pod;
      if (r >= 0) {
        const int32_t id = idx.ident(p);
        placed.push_back(Placed{r, id, idx.aclass(p, false)});
      } else if (has_pod_affinity(p)) {
        // the reference's metadata then errs on the node-less NodeInfo (predicates/metadata.go:106-109)
        fail(KSIM_E_UNSUPPORTED, "a pod with inter-pod affinity terms cached on a node that is not listed");
      }
    }
  }
  std::vector<const Labels*> labels;
  for (const Str& n : c->names) labels.push_back(&c->infos[n].node.labels);
  AffTables t;
  build_aff_tables(idx, labels, placed, false, &t);
  check(c, load_aff_tab(t, (int64_t)c->names.size(), c->opt.hard_weight, c->h), "ksim_load_affinity");
  c->aff_remap = t.remap;
  c->aff_sig = aff_signature(idx);
  c->have_sig = true;
  c->aff_check = false;
  c->stats[0] += 1;
}

// SchedulerCache._sync_affinity: the pod's aff_ident / aff_class against tables kept current.
void sync_affinity(Cache* c, Enc* e, const PodObj& p) {
  if (!c->aff_wanted) return;
  if (!c->aff_on) {
    if (!has_pod_affinity(p) && p.spread.empty()) return;
    c->aff_on = true;
  }
  int32_t me_ident = 0, me_class = -1;
  for (int attempt = 0; attempt < 2; ++attempt) {
    const bool fresh = !c->aidx;
    if (fresh) {
      c->aidx.reset(new AffinityIndex());
      c->aidx->hard_weight = c->opt.hard_weight;
      c->have_sig = false;
    }
    AffinityIndex& idx = *c->aidx;
    me_ident = idx.ident(p);
    me_class = idx.aclass(p, true);
    if (c->have_sig && !c->aff_check && grew_only_dead(c, idx)) {
      c->aff_remap.resize(idx.idents.items.size(), 0);
      c->aff_sig = aff_signature(idx);
      break;
    }
    try {
      aff_rebuild(c, idx);
      break;
    } catch (const Fail& f) {
      // a long-lived index keeps every selector / term it has seen: retry from the live pods
      if (f.code != KSIM_E_UNSUPPORTED || fresh || attempt) throw;
      c->aidx.reset();
    }
  }
  e->row.aff_ident = c->aff_remap[me_ident];
  e->row.aff_class = me_class + 1;
}

// ---------------------------------------------------------------- node rows
struct RowBuf {
  ksim_node_row row{};
  int64_t alloc_s[KSIM_MAX_SCALAR] = {}, req_s[KSIM_MAX_SCALAR] = {};
  std::vector<uint64_t> ports;
};

// NodeInfo.SetNode's columns + the dynamic columns of the pods the NodeInfo holds.
void node_row(Cache* c, const NodeObj& x, const Info& info, Str* mem, Str* disk, RowBuf* b) {
  const int32_t lid = c->in.label_set(x);
  const int32_t tid = c->in.taint_sets.get(x.taints);
  for (const auto& o : x.other)
    if (is_scalar_resource(o.first)) b->alloc_s[scalar_id(c, o.first)] = o.second;
  load_tables(c);
  ksim_node_row& r = b->row;
  r.alloc_cpu = x.alloc[0]; r.alloc_mem = x.alloc[1]; r.alloc_gpu = x.alloc[2]; r.alloc_eph = x.alloc[3];
  r.allowed_pods = (int32_t)x.pods;
  r.flags = node_flags(x, mem, disk);
  if (c->pol_presence)  // CheckNodeLabelPresence (predicates.go:875-910): a function of the label set
    for (const Str& l : c->pol.presence_labels)
      if ((x.labels.count(l) != 0) != c->pol.presence) { r.flags |= KSIM_N_LABEL_PRESENCE; break; }
  r.label_set = lid;
  r.taint_set = tid;
  std::set<uint64_t> seen;
  for (const auto& kv : info.pods) {
    const ksim_pod& d = kv.second.enc.row;
    r.req_cpu += d.add_cpu; r.req_mem += d.add_mem; r.req_gpu += d.add_gpu; r.req_eph += d.add_eph;
    r.nz_cpu += d.nz_cpu; r.nz_mem += d.nz_mem;
    for (const ksim_scalar_req& s : kv.second.enc.scalars) b->req_s[s.col] += s.add;
    for (uint64_t k : kv.second.enc.ports)
      if (seen.insert(k).second) b->ports.push_back(k);
  }
  r.pod_count = (int32_t)info.pods.size();
  r.port_count = (int32_t)b->ports.size();
  r.alloc_scalar = b->alloc_s;
  r.req_scalar = b->req_s;
  r.ports = b->ports.empty() ? nullptr : b->ports.data();
}

void node_event(Cache* c) {  // the device marks its affinity / volume tables stale on node events
  c->vol_dirty = c->vol_loaded;
  c->aidx.reset();
}

void add_node(Cache* c, const NodeObj& x) {
  Info& info = c->infos[x.name];
  Str mem = info.mem, disk = info.disk;
  RowBuf b;
  node_row(c, x, info, &mem, &disk, &b);
  const int64_t r = rank_of(c, x.name);
  if (r >= 0) {
    check(c, ksim_node_update(c->h, r, &b.row), "ksim_node_update");
  } else {
    const int64_t at = std::lower_bound(c->names.begin(), c->names.end(), x.name) - c->names.begin();
    check(c, ksim_node_add(c->h, at, &b.row), "ksim_node_add");
    c->names.insert(c->names.begin() + at, x.name);
    c->rank_valid = false;
  }
  info.has_node = true;
  info.node = x;
  info.mem = mem;
  info.disk = disk;
  node_event(c);
}

void remove_node(Cache* c, const Str& name) {
  const int64_t r = rank_of(c, name);
  if (r < 0) fail(KSIM_E_STATE, "node %s is not in the cache", name.c_str());
  check(c, ksim_node_remove(c->h, r), "ksim_node_remove");
  c->names.erase(c->names.begin() + r);
  c->rank_valid = false;
  Info& info = c->infos[name];
  info.has_node = false;
  info.node = NodeObj();
  info.mem = info.disk = "Unknown";
  if (info.pods.empty()) c->infos.erase(name);
  node_event(c);
}

// ---------------------------------------------------------------- pods (cache.go:200-228)
void pod_args(const Enc& e, const uint64_t** pp, int32_t* np, const ksim_scalar_req** sp, int32_t* ns) {
  *pp = e.ports.empty() ? nullptr : e.ports.data();
  *np = (int32_t)e.ports.size();
  *sp = e.scalars.empty() ? nullptr : e.scalars.data();
  *ns = (int32_t)e.scalars.size();
}

void add(Cache* c, const PodObj& p, Enc e) {
  const Str& name = p.node_name;
  const int64_t r = rank_of(c, name);
  if (r >= 0) {
    sync_volumes(c, e.row.vol_class != 0, &e);
    sync_affinity(c, &e, p);
    const uint64_t* pp; const ksim_scalar_req* sp; int32_t np, ns;
    pod_args(e, &pp, &np, &sp, &ns);
    check(c, ksim_pod_add(c->h, r, &e.row, pp, np, sp, ns), "ksim_pod_add");
  } else if (c->aff_on) {
    c->aff_check = true;
  }
  Info& info = c->infos[name];
  mount(c, name, e, 1);
  info.pods[pod_key(p)] = PodRec{p, std::move(e)};
}

void remove(Cache* c, const PodObj& p) {
  const Str& name = p.node_name;
  const Str key = pod_key(p);
  auto it = c->infos.find(name);
  if (it == c->infos.end() || !it->second.pods.count(key))
    fail(KSIM_E_STATE, "no corresponding pod %s in pods of node %s", p.name.c_str(), name.c_str());
  PodRec& rec = it->second.pods[key];
  const int64_t r = rank_of(c, name);
  if (r >= 0) {
    sync_volumes(c, rec.enc.row.vol_class != 0, nullptr);
    sync_affinity(c, &rec.enc, rec.pod);
    const uint64_t* pp; const ksim_scalar_req* sp; int32_t np, ns;
    pod_args(rec.enc, &pp, &np, &sp, &ns);
    check(c, ksim_pod_remove(c->h, r, &rec.enc.row, pp, np, sp, ns), "ksim_pod_remove");
  }
  const Enc e = rec.enc;
  it->second.pods.erase(key);
  mount(c, name, e, -1);
  if (it->second.pods.empty() && !it->second.has_node) c->infos.erase(it);
}

bool cache_profile() {
  static const bool on = getenv("KSIM_CACHE_PROFILE") && atoi(getenv("KSIM_CACHE_PROFILE")) != 0;
  return on;
}

int64_t profile_skip() {
  static const int64_t k = getenv("KSIM_CACHE_PROFILE_SKIP") ? atoll(getenv("KSIM_CACHE_PROFILE_SKIP")) : 0;
  return k;
}

struct PhaseClock {
  Cache* c;
  bool on;
  std::chrono::steady_clock::time_point t;
  explicit PhaseClock(Cache* cc) : c(cc), on(cache_profile() && cc->prof_seen++ >= profile_skip()) {
    if (on) t = std::chrono::steady_clock::now();
  }
  void lap(int k) {
    if (!on) return;
    const auto now = std::chrono::steady_clock::now();
    c->prof[k] += std::chrono::duration_cast<std::chrono::nanoseconds>(now - t).count();
    t = now;
  }
};

void schedule(Cache* c, PodObj p, int32_t assume, ksim_result* out) {
  PhaseClock pc(c);
  if (pc.on) c->prof[6] += 1;
  Enc e = encode(c, p);
  pc.lap(0);
  if (has_pred_volumes(p)) check_volume_errors(c, p);
  pc.lap(1);
  sync_volumes(c, e.row.vol_class != 0, &e);
  pc.lap(2);
  sync_affinity(c, &e, p);
  pc.lap(3);
  const Str key = pod_key(p);
  // Scheduler.assume runs after Schedule: a pod already in the cache is decided (lastNodeIndex moves)
  // and then refused by AssumePod
  const bool dup = assume && c->pod_states.count(key);
  const uint64_t* pp; const ksim_scalar_req* sp; int32_t np, ns;
  pod_args(e, &pp, &np, &sp, &ns);
  const int rc = ksim_schedule_one(c->h, &e.row, pp, np, sp, ns, assume && !dup ? KSIM_SCHEDULE_ASSUME : KSIM_SCHEDULE_ONLY, out);
  pc.lap(4);
  if (rc == KSIM_E_NO_NODES) fail(rc, "no nodes available to schedule pods");
  check(c, rc, "ksim_schedule_one");
  if (out->node < 0 || !assume) return;
  if (dup) fail(KSIM_E_STATE, "pod %s is in the cache, so can't be assumed", key.c_str());
  // the device already holds the commit: record it host-side with the assumed pod's encoding
  const Str& host = c->names[out->node];
  p.node_name = host;  // (the call's own copy: moved into the cache below)
  e.row.host = out->node;
  Info& info = c->infos[host];
  mount(c, host, e, 1);
  c->pod_states[key] = p;
  c->assumed.insert(key);
  info.pods[key] = PodRec{std::move(p), std::move(e)};
  pc.lap(5);
}

}  // namespace

// ---------------------------------------------------------------- C-ABI
static Str g_create_err = "null cache";  // ksim_k8s_cache_last_error(NULL): why the last create failed

extern "C" int ksim_k8s_cache_create(const ksim_k8s_cache_options* opt, ksim_k8s_cache** out) {
  if (!opt || !out) return KSIM_E_INVAL;
  *out = nullptr;
  auto* c = new ksim_k8s_cache();
  c->opt = *opt;
  if (c->opt.port_slots <= 0) c->opt.port_slots = 8;
  default_max_vols(c->opt.max_vols);
  const int rc = guard(c, [&] {
    const ksim_config& cfg = c->opt.cfg;
    const uint32_t pr = cfg.predicates;
    if (const ksim_k8s_policy_args* a = c->opt.policy) {
      PolicyArgs& pol = c->pol;
      pol.on = true;
      for (int32_t i = 0; i < a->n_presence_labels; ++i) pol.presence_labels.push_back(S(a->presence_labels[i]));
      pol.presence = a->presence != 0;
      for (int32_t i = 0; i < a->n_affinity_labels; ++i) pol.affinity_labels.push_back(S(a->affinity_labels[i]));
      for (int32_t i = 0; i < a->n_label_priorities; ++i) {
        if (a->label_priorities[i].weight <= 0) fail(KSIM_E_INVAL, "label priority: weight must be positive");
        pol.label_prios.push_back({S(a->label_priorities[i].label),
                                   {a->label_priorities[i].presence != 0, a->label_priorities[i].weight}});
      }
      if (a->n_label_priorities > 0 && cfg.no_priorities)
        fail(KSIM_E_INVAL, "label priorities are prioritizers: cfg.no_priorities must be 0 when n_label_priorities > 0");
      if (a->services_select_pods && ((pr & KSIM_P_SERVICE_AFFINITY) || a->has_service_anti_affinity))
        fail(KSIM_E_UNSUPPORTED, "CheckServiceAffinity / serviceAntiAffinity with services selecting the pods (the Python "
                                 "host builds their service-aware tables)");
      c->opt.policy = nullptr;  // copied
      c->pol_presence = (pr & KSIM_P_LABEL_PRESENCE) != 0;
      c->pol_svc = (pr & KSIM_P_SERVICE_AFFINITY) != 0;
    } else if (pr & (KSIM_P_LABEL_PRESENCE | KSIM_P_SERVICE_AFFINITY)) {
      fail(KSIM_E_UNSUPPORTED, "CheckNodeLabelPresence / CheckServiceAffinity need their Policy arguments "
                               "(ksim_k8s_cache_options.policy)");
    }
    c->need_na = cfg.weights[KSIM_W_NODE_AFFINITY] != 0;
    c->aff_wanted = (pr & KSIM_P_INTERPOD_AFFINITY) ||
                    ((cfg.weights[KSIM_W_INTERPOD_AFFINITY] || cfg.weights[KSIM_W_SELECTOR_SPREAD]) && !cfg.no_priorities);
    c->vol_on = (pr & VOLUME_BITS) != 0;
    c->use_zone = (pr & KSIM_P_VOLUME_ZONE) != 0;
    c->in.images = c->opt.extra.image_locality != 0;
    check(c, ksim_create(&cfg, &c->h), "ksim_create");
    c->in.label_sets.get(LabelSetKey{});
    c->in.taint_sets.get({});
    c->in.classes.get(class_key(PodObj{}, c->in.images));
    load_tables(c);
    ksim_node_table t{};  // scalar columns reserved up front: new names need no relayout
    t.n_nodes = 0;
    t.n_scalar = KSIM_MAX_SCALAR;
    t.port_slots = c->opt.port_slots;
    check(c, ksim_load_nodes(c->h, &t), "ksim_load_nodes");
  });
  if (rc) {
    if (c->h) ksim_destroy(c->h);
    g_create_err = c->err;
    delete c;
    return rc;
  }
  *out = c;
  return KSIM_OK;
}

extern "C" void ksim_k8s_cache_destroy(ksim_k8s_cache* c) {
  if (!c) return;
  if (cache_profile() && c->prof[6])
    fprintf(stderr, "[ksim cache profile] %lld Schedule calls, us/call: encode %.1f volume-errors %.1f volume-sync %.1f "
            "affinity-sync %.1f schedule_one %.1f bookkeeping %.1f\n", (long long)c->prof[6], c->prof[0] / 1e3 / c->prof[6],
            c->prof[1] / 1e3 / c->prof[6], c->prof[2] / 1e3 / c->prof[6], c->prof[3] / 1e3 / c->prof[6],
            c->prof[4] / 1e3 / c->prof[6], c->prof[5] / 1e3 / c->prof[6]);
  if (c->h) ksim_destroy(c->h);
  delete c;
}

extern "C" const char* ksim_k8s_cache_last_error(const ksim_k8s_cache* c) { return c ? c->err.c_str() : g_create_err.c_str(); }

extern "C" int ksim_k8s_cache_add_pv(ksim_k8s_cache* c, const ksim_k8s_pv* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] { add_pv(&c->vidx, *x); });
}

extern "C" int ksim_k8s_cache_add_pvc(ksim_k8s_cache* c, const ksim_k8s_pvc* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] { add_pvc(&c->vidx, *x); });
}

extern "C" int ksim_k8s_cache_add_storage_class(ksim_k8s_cache* c, const ksim_k8s_storage_class* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] { add_storage_class(&c->vidx, *x); });
}

extern "C" int ksim_k8s_cache_add_node(ksim_k8s_cache* c, const ksim_k8s_node* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] { add_node(c, copy_node(*x)); });
}

extern "C" int ksim_k8s_cache_update_node(ksim_k8s_cache* c, const ksim_k8s_node* old_node, const ksim_k8s_node* x) {
  (void)old_node;  // cache.UpdateNode reads only the new object
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] { add_node(c, copy_node(*x)); });
}

extern "C" int ksim_k8s_cache_remove_node(ksim_k8s_cache* c, const ksim_k8s_node* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] { remove_node(c, S(x->name)); });
}

extern "C" int ksim_k8s_cache_assume_pod(ksim_k8s_cache* c, const ksim_k8s_pod* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] {
    const PodObj p = copy_pod(*x);
    const Str key = pod_key(p);
    if (c->pod_states.count(key)) fail(KSIM_E_STATE, "pod %s is in the cache, so can't be assumed", key.c_str());
    add(c, p, encode(c, p));
    c->pod_states[key] = p;
    c->assumed.insert(key);
  });
}

extern "C" int ksim_k8s_cache_forget_pod(ksim_k8s_cache* c, const ksim_k8s_pod* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] {
    const PodObj p = copy_pod(*x);
    const Str key = pod_key(p);
    auto cur = c->pod_states.find(key);
    if (cur != c->pod_states.end() && cur->second.node_name != p.node_name)
      fail(KSIM_E_STATE, "pod %s was assumed on %s but assigned to %s", key.c_str(), p.node_name.c_str(), cur->second.node_name.c_str());
    if (cur == c->pod_states.end() || !c->assumed.count(key))
      fail(KSIM_E_STATE, "pod %s wasn't assumed so cannot be forgotten", key.c_str());
    remove(c, p);
    c->assumed.erase(key);
    c->pod_states.erase(key);
  });
}

extern "C" int ksim_k8s_cache_add_pod(ksim_k8s_cache* c, const ksim_k8s_pod* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] {
    const PodObj p = copy_pod(*x);
    const Str key = pod_key(p);
    auto cur = c->pod_states.find(key);
    if (cur != c->pod_states.end() && c->assumed.count(key)) {
      if (cur->second.node_name != p.node_name) {  // the binding landed elsewhere
        remove(c, cur->second);
        add(c, p, encode(c, p));
      }
      c->assumed.erase(key);
      c->pod_states[key] = p;
    } else if (cur == c->pod_states.end()) {
      add(c, p, encode(c, p));
      c->pod_states[key] = p;
    } else {
      fail(KSIM_E_STATE, "pod %s was already in added state", key.c_str());
    }
  });
}

extern "C" int ksim_k8s_cache_update_pod(ksim_k8s_cache* c, const ksim_k8s_pod* old_pod, const ksim_k8s_pod* new_pod) {
  if (!c || !old_pod || !new_pod) return KSIM_E_INVAL;
  return guard(c, [&] {
    const PodObj o = copy_pod(*old_pod), n = copy_pod(*new_pod);
    const Str key = pod_key(o);
    if (!c->pod_states.count(key) || c->assumed.count(key))
      fail(KSIM_E_STATE, "pod %s is not added to scheduler cache, so cannot be updated", key.c_str());
    remove(c, o);
    add(c, n, encode(c, n));
    c->pod_states[key] = n;
  });
}

extern "C" int ksim_k8s_cache_remove_pod(ksim_k8s_cache* c, const ksim_k8s_pod* x) {
  if (!c || !x) return KSIM_E_INVAL;
  return guard(c, [&] {
    const PodObj p = copy_pod(*x);
    const Str key = pod_key(p);
    auto cur = c->pod_states.find(key);
    if (cur == c->pod_states.end() || c->assumed.count(key))
      fail(KSIM_E_STATE, "pod %s is not found in scheduler cache, so cannot be removed from it", key.c_str());
    remove(c, cur->second);
    c->pod_states.erase(key);
  });
}

extern "C" int ksim_k8s_cache_schedule(ksim_k8s_cache* c, const ksim_k8s_pod* x, int32_t assume, ksim_result* out) {
  if (!c || !x || !out) return KSIM_E_INVAL;
  return guard(c, [&] { schedule(c, copy_pod(*x), assume, out); });
}

extern "C" int32_t ksim_k8s_cache_fit_error(const ksim_k8s_cache* c, const ksim_result* res, char* buf, int32_t cap) {
  if (!c || !res) return -1;
  const Str s = fit_error_text((int64_t)c->names.size(), res->reasons, c->in.scalar_names.items);
  if (buf && cap > 0) {
    const size_t k = std::min<size_t>(s.size(), (size_t)cap - 1);
    memcpy(buf, s.data(), k);
    buf[k] = 0;
  }
  return (int32_t)s.size();
}

extern "C" int64_t ksim_k8s_cache_node_count(const ksim_k8s_cache* c) { return c ? (int64_t)c->names.size() : -1; }

extern "C" const char* ksim_k8s_cache_node_name(const ksim_k8s_cache* c, int64_t rank) {
  if (!c || rank < 0 || rank >= (int64_t)c->names.size()) return nullptr;
  return c->names[rank].c_str();
}

extern "C" ksim_handle* ksim_k8s_cache_handle(ksim_k8s_cache* c) { return c ? c->h : nullptr; }

extern "C" int ksim_k8s_cache_stats(const ksim_k8s_cache* c, int64_t* out4) {
  if (!c || !out4) return KSIM_E_INVAL;
  for (int k = 0; k < 4; ++k) out4[k] = c->stats[k];
  return KSIM_OK;
}
