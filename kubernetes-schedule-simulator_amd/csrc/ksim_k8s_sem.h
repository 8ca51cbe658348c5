// ksim_k8s_sem.h — the Kubernetes semantics shared by the snapshot front end (ksim_k8s.cpp) and the
// event-driven scheduler cache (ksim_k8s_cache.cpp): label selectors, node selectors and node
// affinity, tolerations, request vectors, the interning of label / taint sets, pod classes, inter-pod
// affinity identities and terms, volume identities, and the table builders over them.  Everything is
// in an anonymous namespace: each translation unit that includes it has its own copy.
//
// Reference semantics (paths under vendor/k8s.io/; S/ = kubernetes/pkg/scheduler/):
//  - label selectors: apimachinery/pkg/labels/selector.go:193-235 (Requirement.Matches), :837-853
//    (SelectorFromSet), NewRequirement's validation (:124-170), validation.IsQualifiedName /
//    IsValidLabelValue (apimachinery/pkg/util/validation/validation.go:34-112);
//    metav1.LabelSelectorAsSelector (apimachinery/pkg/apis/meta/v1/helpers.go:31-70);
//    NodeSelectorRequirementsAsSelector (kubernetes/pkg/apis/core/v1/helper/helpers.go:215-245);
//  - podMatchesNodeLabels / nodeMatchesNodeSelectorTerms: S/algorithm/predicates/predicates.go:780-838;
//  - PodToleratesNodeTaints / ToleratesTaint: predicates.go:1465-1494, api/core/v1/toleration.go:37-56;
//  - TaintToleration / NodeAffinity map values: S/algorithm/priorities/taint_toleration.go:29-73,
//    node_affinity.go:34-75; NodePreferAvoidPods: node_prefer_avoid_pods.go:32-68; ImageLocality:
//    image_locality.go:39-88;
//  - NodeInfo.SetNode / AddPod, calculateResource: S/schedulercache/node_info.go:318-448;
//    GetResourceRequest: predicates.go:659-697; GetNonzeroRequests: priorities/util/non_zero.go:38-53;
//    CheckNodeConditionPredicate: predicates.go:1534-1568; HostPortInfo: S/util/utils.go:31-155;
//  - inter-pod affinity: predicates.go:1143-1450, priorities/interpod_affinity.go:118-240,
//    priorities/util/topologies.go:28-71; SelectorSpread zones: utilnode.GetZoneKey;
//  - volumes: predicates.go:220-285 (NoDiskConflict), :287-507 (MaxPD), :539-633 (VolumeZone).
// The table layouts and the interning rules are the Python host's (ksim/ingest.py, labels.py,
// affinity.py, volumes.py, scheduler.py), which tests/test_k8s_frontend.py compares with.
#ifndef KSIM_K8S_SEM_H
#define KSIM_K8S_SEM_H

#include <algorithm>
#include <array>
#include <cerrno>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <set>
#include <string>
#include <tuple>
#include <vector>

#include "../../include/ksim_k8s.h"

namespace {

using Str = std::string;
using Labels = std::map<Str, Str>;

Str S(const char* p) { return p ? Str(p) : Str(); }

struct Fail {
  int code;
  Str msg;
};

[[noreturn]] void fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  throw Fail{code, buf};
}

// ---------------------------------------------------------------- labels (ksim/labels.py)
bool alnum(char c) { return (c >= 'a' && c <= 'z') || (c >= 'A' && c <= 'Z') || (c >= '0' && c <= '9'); }

// (?:[A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]
bool name_re(const Str& s) {
  if (s.empty() || !alnum(s.front()) || !alnum(s.back())) return false;
  for (char c : s)
    if (!alnum(c) && c != '-' && c != '_' && c != '.') return false;
  return true;
}

// DNS-1123 subdomain: [a-z0-9]([-a-z0-9]*[a-z0-9])?(\.[a-z0-9]([-a-z0-9]*[a-z0-9])?)*
bool dns_subdomain(const Str& s) {
  if (s.empty()) return false;
  size_t i = 0;
  for (;;) {
    size_t j = s.find('.', i);
    const Str part = s.substr(i, j == Str::npos ? Str::npos : j - i);
    if (part.empty()) return false;
    auto lo = [](char c) { return (c >= 'a' && c <= 'z') || (c >= '0' && c <= '9'); };
    if (!lo(part.front()) || !lo(part.back())) return false;
    for (char c : part)
      if (!lo(c) && c != '-') return false;
    if (j == Str::npos) return true;
    i = j + 1;
  }
}

bool qualified_name(const Str& k) {
  const size_t n = std::count(k.begin(), k.end(), '/');
  if (n > 1) return false;
  Str name = k;
  if (n == 1) {
    const size_t p = k.find('/');
    const Str prefix = k.substr(0, p);
    name = k.substr(p + 1);
    if (prefix.empty() || prefix.size() > 253 || !dns_subdomain(prefix)) return false;
  }
  return !name.empty() && name.size() <= 63 && name_re(name);
}

bool label_value_ok(const Str& v) { return v.size() <= 63 && (v.empty() || name_re(v)); }

bool parse_i64(const Str& s, int64_t* out) {
  size_t i = 0;
  if (i < s.size() && (s[i] == '+' || s[i] == '-')) ++i;
  if (i == s.size()) return false;
  for (size_t k = i; k < s.size(); ++k)
    if (s[k] < '0' || s[k] > '9') return false;
  errno = 0;
  char* end = nullptr;
  const long long v = strtoll(s.c_str(), &end, 10);
  if (errno == ERANGE) return false;
  *out = v;
  return true;
}

enum Op { OP_IN, OP_NOTIN, OP_EXISTS, OP_DNE, OP_GT, OP_LT };

struct Req {
  Str key;
  Str op;  // as spelled (validation and the interning key)
  Op o;
  std::vector<Str> vals;  // sorted
  bool operator<(const Req& r) const { return std::tie(key, op, vals) < std::tie(r.key, r.op, r.vals); }
  bool operator==(const Req& r) const { return key == r.key && op == r.op && vals == r.vals; }
};

// A selector: nothing = matches no label set (labels.Nothing()); otherwise an AND of requirements.
struct Sel {
  bool nothing = false;
  std::vector<Req> reqs;
  bool operator<(const Sel& s) const { return std::tie(nothing, reqs) < std::tie(s.nothing, s.reqs); }
  bool operator==(const Sel& s) const { return nothing == s.nothing && reqs == s.reqs; }
};

// labels.NewRequirement with its validation; false on an error.
bool requirement(const Str& key, const Str& op, std::vector<Str> vals, Req* out) {
  if (!qualified_name(key)) return false;
  Op o;
  if (op == "In" || op == "NotIn") {
    if (vals.empty()) return false;
    o = op == "In" ? OP_IN : OP_NOTIN;
  } else if (op == "=" || op == "==" || op == "!=") {
    if (vals.size() != 1) return false;
    o = op == "!=" ? OP_NOTIN : OP_IN;
  } else if (op == "Exists" || op == "DoesNotExist") {
    if (!vals.empty()) return false;
    o = op == "Exists" ? OP_EXISTS : OP_DNE;
  } else if (op == "Gt" || op == "Lt") {
    int64_t x;
    if (vals.size() != 1 || !parse_i64(vals[0], &x)) return false;
    o = op == "Gt" ? OP_GT : OP_LT;
  } else {
    return false;
  }
  for (const Str& v : vals)
    if (!label_value_ok(v)) return false;
  std::sort(vals.begin(), vals.end());
  *out = Req{key, op, o, vals};
  return true;
}

bool req_matches(const Req& r, const Labels& lab) {
  auto it = lab.find(r.key);
  const bool has = it != lab.end();
  switch (r.o) {
    case OP_IN: return has && std::binary_search(r.vals.begin(), r.vals.end(), it->second);
    case OP_NOTIN: return !has || !std::binary_search(r.vals.begin(), r.vals.end(), it->second);
    case OP_EXISTS: return has;
    case OP_DNE: return !has;
    case OP_GT:
    case OP_LT: {
      if (!has || r.vals.size() != 1) return false;
      int64_t lv, rv;
      if (!parse_i64(it->second, &lv) || !parse_i64(r.vals[0], &rv)) return false;
      return r.o == OP_GT ? lv > rv : lv < rv;
    }
  }
  return false;
}

bool matches(const Sel& s, const Labels& lab) {
  if (s.nothing) return false;
  for (const Req& r : s.reqs)
    if (!req_matches(r, lab)) return false;
  return true;
}

// SelectorFromSet: an invalid key / value makes the selector Everything().
Sel from_set(const std::vector<std::pair<Str, Str>>& kv) {
  Sel s;
  for (const auto& e : kv) {
    Req r;
    if (!requirement(e.first, "=", {e.second}, &r)) return Sel{};
    s.reqs.push_back(r);
  }
  return s;
}

std::vector<Str> strs(int32_t n, const char* const* p) {
  std::vector<Str> v;
  for (int32_t i = 0; i < n; ++i) v.push_back(S(p[i]));
  return v;
}

// NodeSelectorRequirementsAsSelector: Nothing for an empty list; false on an error.
bool from_node_reqs(const std::vector<Req>& raw, Sel* out) {
  if (raw.empty()) {
    *out = Sel{true, {}};
    return true;
  }
  Sel s;
  for (const Req& e : raw) {
    if (e.op != "In" && e.op != "NotIn" && e.op != "Exists" && e.op != "DoesNotExist" && e.op != "Gt" && e.op != "Lt")
      return false;
    Req r;
    if (!requirement(e.key, e.op, e.vals, &r)) return false;
    s.reqs.push_back(r);
  }
  *out = s;
  return true;
}

// Raw requirement lists as passed (unvalidated, values unsorted).
std::vector<Req> raw_reqs(int32_t n, const ksim_k8s_req* r) {
  std::vector<Req> v;
  for (int32_t i = 0; i < n; ++i) v.push_back(Req{S(r[i].key), S(r[i].op), OP_IN, strs(r[i].n_values, r[i].values)});
  return v;
}

struct LabelSel {  // a metav1.LabelSelector as passed
  bool present = false;
  std::vector<std::pair<Str, Str>> ml;
  std::vector<Req> exprs;
};

LabelSel copy_ls(const ksim_k8s_label_selector& x) {
  LabelSel s;
  s.present = x.present != 0;
  for (int32_t i = 0; i < x.n_match_labels; ++i) s.ml.push_back({S(x.match_labels[i].key), S(x.match_labels[i].value)});
  s.exprs = raw_reqs(x.n_exprs, x.exprs);
  return s;
}

// LabelSelectorAsSelector: nil → Nothing, empty → Everything; false on an error.
bool from_label_selector(const LabelSel& ls, Sel* out) {
  if (!ls.present) {
    *out = Sel{true, {}};
    return true;
  }
  Sel s;
  if (ls.ml.empty() && ls.exprs.empty()) {
    *out = s;
    return true;
  }
  std::map<Str, Str> ml;
  for (const auto& e : ls.ml) ml[e.first] = e.second;  // a Go map: the last duplicate wins
  for (const auto& e : ml) {
    Req r;
    if (!requirement(e.first, "=", {e.second}, &r)) return false;
    s.reqs.push_back(r);
  }
  for (const Req& e : ls.exprs) {
    if (e.op != "In" && e.op != "NotIn" && e.op != "Exists" && e.op != "DoesNotExist") return false;
    Req r;
    if (!requirement(e.key, e.op, e.vals, &r)) return false;
    s.reqs.push_back(r);
  }
  *out = s;
  return true;
}

// ---------------------------------------------------------------- object copies
struct Taint {
  Str key, value, effect;
  bool operator<(const Taint& t) const { return std::tie(key, value, effect) < std::tie(t.key, t.value, t.effect); }
  bool operator==(const Taint& t) const { return key == t.key && value == t.value && effect == t.effect; }
};
struct Tol {
  Str key, op, value, effect;
  bool operator<(const Tol& t) const { return std::tie(key, op, value, effect) < std::tie(t.key, t.op, t.value, t.effect); }
};

bool tolerates(const Tol& t, const Taint& x) {
  if (!t.effect.empty() && t.effect != x.effect) return false;
  if (!t.key.empty() && t.key != x.key) return false;
  if (t.op.empty() || t.op == "Equal") return t.value == x.value;
  return t.op == "Exists";
}

struct Avoid {
  bool has = false;
  Str kind, uid;
  bool operator<(const Avoid& a) const { return std::tie(has, kind, uid) < std::tie(a.has, a.kind, a.uid); }
};

struct NodeObj {
  Str name;
  Labels labels;
  std::vector<Taint> taints;
  bool unschedulable = false;
  std::vector<std::pair<Str, Str>> conds;
  int64_t alloc[4] = {0, 0, 0, 0};
  int64_t pods = 0;
  std::vector<std::pair<Str, int64_t>> other;
  std::vector<Avoid> avoid;
  bool has_images = false;                          // status.images is non-empty
  std::vector<std::pair<Str, int64_t>> images;      // totalImageSize's map: name -> size (sorted)
};

struct Container {
  bool has_cpu = false, has_mem = false;
  int64_t cpu = 0, mem = 0, gpu = 0, eph = 0;
  std::vector<std::pair<Str, int64_t>> other;
  bool qos = false;
  std::vector<std::tuple<Str, Str, int32_t>> ports;
  Str image;
};

struct PodTerm {
  LabelSel sel;
  std::vector<Str> nss;
  Str key;
  int32_t weight = 0;
};

struct Volume {
  int32_t kind = 0;
  bool ro = false;
  Str id, pool, image;
  std::vector<Str> monitors;
};

struct NodeAff {
  bool has = false, has_required = false;
  std::vector<std::vector<Req>> required;              // raw terms
  std::vector<std::pair<int32_t, std::vector<Req>>> preferred;
};

struct PodObj {
  Str name, ns, uid;
  Labels labels;
  bool deleting = false;
  Str node_name;
  std::vector<Container> cs, init;
  std::vector<std::pair<Str, Str>> node_selector;
  NodeAff na;
  std::vector<Tol> tols;
  bool has_pa = false, has_anti = false;
  std::vector<PodTerm> a_req, a_pref, n_req, n_pref;
  std::vector<Volume> vols;
  std::vector<Sel> spread;  // resolved SelectorSpread selectors
  bool has_ctrl = false;
  Str ctrl_kind, ctrl_uid;
};

std::vector<PodTerm> copy_terms(int32_t n, const ksim_k8s_pod_term* t) {
  std::vector<PodTerm> v;
  for (int32_t i = 0; i < n; ++i) {
    PodTerm x;
    x.sel = copy_ls(t[i].selector);
    x.nss = strs(t[i].n_namespaces, t[i].namespaces);
    x.key = S(t[i].topology_key);
    x.weight = t[i].weight;
    v.push_back(x);
  }
  return v;
}

Container copy_container(const ksim_k8s_container& c) {
  Container x;
  x.has_cpu = c.has_cpu != 0;
  x.has_mem = c.has_mem != 0;
  x.cpu = c.cpu_milli; x.mem = c.mem; x.gpu = c.gpu; x.eph = c.eph;
  for (int32_t i = 0; i < c.n_other; ++i) x.other.push_back({S(c.other[i].name), c.other[i].value});
  x.qos = c.qos_positive != 0;
  for (int32_t i = 0; i < c.n_ports; ++i)
    x.ports.emplace_back(S(c.ports[i].host_ip), S(c.ports[i].protocol), c.ports[i].host_port);
  x.image = S(c.image);
  return x;
}

PodObj copy_pod(const ksim_k8s_pod& p) {
  PodObj o;
  o.name = S(p.name);
  o.ns = S(p.namespace_);
  o.uid = S(p.uid);
  for (int32_t i = 0; i < p.n_labels; ++i) o.labels[S(p.labels[i].key)] = S(p.labels[i].value);
  o.deleting = p.deleting != 0;
  o.node_name = S(p.node_name);
  for (int32_t i = 0; i < p.n_containers; ++i) o.cs.push_back(copy_container(p.containers[i]));
  for (int32_t i = 0; i < p.n_init_containers; ++i) o.init.push_back(copy_container(p.init_containers[i]));
  {
    std::map<Str, Str> ns;  // a Go map
    for (int32_t i = 0; i < p.n_node_selector; ++i) ns[S(p.node_selector[i].key)] = S(p.node_selector[i].value);
    o.node_selector.assign(ns.begin(), ns.end());
  }
  o.na.has = p.has_node_affinity != 0;
  o.na.has_required = p.has_required != 0;
  for (int32_t i = 0; i < p.n_required_terms; ++i)
    o.na.required.push_back(raw_reqs(p.required_terms[i].n_reqs, p.required_terms[i].reqs));
  for (int32_t i = 0; i < p.n_preferred; ++i)
    o.na.preferred.push_back({p.preferred[i].weight, raw_reqs(p.preferred[i].preference.n_reqs, p.preferred[i].preference.reqs)});
  for (int32_t i = 0; i < p.n_tolerations; ++i)
    o.tols.push_back(Tol{S(p.tolerations[i].key), S(p.tolerations[i].op), S(p.tolerations[i].value), S(p.tolerations[i].effect)});
  o.has_pa = p.has_pod_affinity != 0;
  o.has_anti = p.has_pod_anti_affinity != 0;
  o.a_req = copy_terms(p.n_affinity_required, p.affinity_required);
  o.a_pref = copy_terms(p.n_affinity_preferred, p.affinity_preferred);
  o.n_req = copy_terms(p.n_anti_required, p.anti_required);
  o.n_pref = copy_terms(p.n_anti_preferred, p.anti_preferred);
  for (int32_t i = 0; i < p.n_volumes; ++i) {
    const ksim_k8s_volume& v = p.volumes[i];
    o.vols.push_back(Volume{v.kind, v.read_only != 0, S(v.id), S(v.pool), S(v.image), strs(v.n_monitors, v.monitors)});
  }
  for (int32_t i = 0; i < p.n_spread; ++i) {
    const LabelSel ls = copy_ls(p.spread[i]);
    Sel s;
    if (p.spread_set_selector && p.spread_set_selector[i]) {
      s = from_set(ls.ml);
    } else if (!from_label_selector(ls, &s)) {
      continue;  // the caller's lister resolution keeps only parsable selectors
    }
    o.spread.push_back(s);
  }
  if (p.avoid_ctrl_kind) {
    o.has_ctrl = true;
    o.ctrl_kind = S(p.avoid_ctrl_kind);
    o.ctrl_uid = S(p.avoid_ctrl_uid);
  }
  return o;
}

// ---------------------------------------------------------------- scheduling semantics
bool pod_matches_node_labels(const PodObj& p, const Labels& lab) {
  if (!p.node_selector.empty() && !matches(from_set(p.node_selector), lab)) return false;
  if (p.na.has) {
    if (!p.na.has_required) return true;
    for (const auto& t : p.na.required) {
      Sel s;
      if (!from_node_reqs(t, &s)) return false;
      if (matches(s, lab)) return true;
    }
    return false;
  }
  return true;
}

// CalculateNodeAffinityPriorityMap's count; false when a preferred term does not parse.
bool preferred_weight(const PodObj& p, const Labels& lab, int64_t* out) {
  int64_t count = 0;
  for (const auto& t : p.na.preferred) {
    if (t.first == 0) continue;
    Sel s;
    if (!from_node_reqs(t.second, &s)) return false;
    if (matches(s, lab)) count += t.first;
  }
  *out = count;
  return true;
}

bool is_scalar_resource(const Str& name) {
  if (name.rfind("hugepages-", 0) == 0) return true;
  if (name.find('/') == Str::npos || name.find("kubernetes.io/") != Str::npos || name.rfind("requests.", 0) == 0)
    return false;
  return qualified_name("requests." + name);
}

struct Res {
  int64_t cpu = 0, mem = 0, gpu = 0, eph = 0;
  std::vector<std::pair<Str, int64_t>> scalar;  // insertion order, presence kept
  int64_t* find(const Str& n) {
    for (auto& e : scalar)
      if (e.first == n) return &e.second;
    return nullptr;
  }
};

struct Compiled {
  Res pred, add;
  int64_t nzc = 0, nzm = 0;
};

// GetResourceRequest / calculateResource / GetNonzeroRequests of one pod.
Compiled container_requests(const PodObj& p) {
  Compiled c;
  for (const Container& x : p.cs) {
    for (Res* r : {&c.pred, &c.add}) {
      r->cpu += x.cpu; r->mem += x.mem; r->gpu += x.gpu; r->eph += x.eph;
      for (const auto& o : x.other) {
        if (!is_scalar_resource(o.first)) continue;
        if (int64_t* v = r->find(o.first)) *v += o.second;
        else r->scalar.push_back(o);
      }
    }
    c.nzc += x.has_cpu ? x.cpu : 100;
    c.nzm += x.has_mem ? x.mem : 200ll * 1024 * 1024;
  }
  for (const Container& x : p.init) {
    c.pred.mem = std::max(c.pred.mem, x.mem);
    c.pred.eph = std::max(c.pred.eph, x.eph);
    c.pred.cpu = std::max(c.pred.cpu, x.cpu);
    c.pred.gpu = std::max(c.pred.gpu, x.gpu);
    for (const auto& o : x.other) {
      if (!is_scalar_resource(o.first)) continue;
      int64_t* v = c.pred.find(o.first);
      if (!v) {
        if (o.second > 0) c.pred.scalar.push_back(o);
      } else if (o.second > *v) {
        *v = o.second;
      }
    }
  }
  return c;
}

bool best_effort(const PodObj& p) {
  for (const Container& x : p.cs)
    if (x.qos) return false;
  return true;
}

std::vector<std::tuple<Str, Str, int32_t>> host_ports(const PodObj& p) {
  std::vector<std::tuple<Str, Str, int32_t>> out;
  for (const Container& x : p.cs)
    for (const auto& e : x.ports) {
      if (std::get<2>(e) <= 0) continue;
      const Str ip = std::get<0>(e).empty() ? "0.0.0.0" : std::get<0>(e);
      const Str proto = std::get<1>(e).empty() ? "TCP" : std::get<1>(e);
      out.emplace_back(ip, proto, std::get<2>(e));
    }
  return out;
}

bool has_pod_affinity(const PodObj& p) { return p.has_pa || p.has_anti; }

bool is_pred_volume(const Volume& v) { return v.kind >= KSIM_K8S_VOL_GCE_PD && v.kind <= KSIM_K8S_VOL_PVC; }

bool has_pred_volumes(const PodObj& p) {
  for (const Volume& v : p.vols)
    if (is_pred_volume(v)) return true;
  return false;
}

// ---------------------------------------------------------------- interning
template <class K>
struct Interner {
  std::map<K, int32_t> ids;
  std::vector<K> items;
  int32_t get(const K& k) {
    auto it = ids.find(k);
    if (it != ids.end()) return it->second;
    const int32_t i = (int32_t)items.size();
    ids.emplace(k, i);
    items.push_back(k);
    return i;
  }
  int32_t find(const K& k) const {
    auto it = ids.find(k);
    return it == ids.end() ? -1 : it->second;
  }
};

// A node label set: its labels, its preferAvoidPods signatures and — when ImageLocality's inputs are
// interned (Interns::images) — its image sizes by name (ingest.label_set_key).
struct LabelSetKey {
  Labels labels;
  std::vector<Avoid> avoid;
  std::vector<std::pair<Str, int64_t>> images;
  bool operator<(const LabelSetKey& o) const {
    return std::tie(labels, avoid, images) < std::tie(o.labels, o.avoid, o.images);
  }
};

// The part of a pod a class stands for: nodeSelector, node affinity, tolerations, RC / RS owner, and
// — when ImageLocality's inputs are interned and some container names an image — the container
// images in order (ingest.pod_class_key).
struct ClassKey {
  std::vector<std::pair<Str, Str>> ns;
  bool na_has = false, na_req = false;
  std::vector<std::vector<Req>> na_required;
  std::vector<std::pair<int32_t, std::vector<Req>>> na_pref;
  std::vector<Tol> tols;
  bool has_ctrl = false;
  Str kind, uid;
  std::vector<Str> images;
  bool operator<(const ClassKey& o) const {
    return std::tie(ns, na_has, na_req, na_required, na_pref, tols, has_ctrl, kind, uid, images) <
           std::tie(o.ns, o.na_has, o.na_req, o.na_required, o.na_pref, o.tols, o.has_ctrl, o.kind, o.uid, o.images);
  }
};

ClassKey class_key(const PodObj& p, bool with_images = false) {
  ClassKey k;
  k.ns = p.node_selector;
  k.na_has = p.na.has;
  k.na_req = p.na.has_required;
  k.na_required = p.na.required;
  k.na_pref = p.na.preferred;
  k.tols = p.tols;
  k.has_ctrl = p.has_ctrl;
  k.kind = p.ctrl_kind;
  k.uid = p.ctrl_uid;
  if (with_images) {  // spec.containers[*].image (init containers are not looked at)
    bool any = false;
    for (const Container& c : p.cs) any |= !c.image.empty();
    if (any)
      for (const Container& c : p.cs) k.images.push_back(c.image);
  }
  return k;
}

PodObj class_pod(const ClassKey& k) {  // the class's pod-side inputs as a pod
  PodObj p;
  p.node_selector = k.ns;
  p.na.has = k.na_has;
  p.na.has_required = k.na_req;
  p.na.required = k.na_required;
  p.na.preferred = k.na_pref;
  p.tols = k.tols;
  p.has_ctrl = k.has_ctrl;
  p.ctrl_kind = k.kind;
  p.ctrl_uid = k.uid;
  return p;
}

constexpr int KEY_ALL = 0, KEY_NODE = 1;
const char* const HOSTNAME = "kubernetes.io/hostname";
const char* const ZONE_KEY = "\x01zone";  // utilnode.GetZoneKey's domains (a pseudo key)

Str zone_key_of(const Labels& lab) {
  auto g = [&](const char* k) {
    auto it = lab.find(k);
    return it == lab.end() ? Str() : it->second;
  };
  const Str region = g("failure-domain.beta.kubernetes.io/region"), zone = g("failure-domain.beta.kubernetes.io/zone");
  if (region.empty() && zone.empty()) return "";
  return region + Str(":\0:", 3) + zone;
}

// ---------------------------------------------------------------- inter-pod affinity (affinity.py)
struct SelItem {  // (namespaces, selector); any_of: a SelectorSpread OR-selector
  std::vector<Str> nss;
  bool any_of = false;
  Sel sel;
  std::vector<Sel> sels;
  bool operator<(const SelItem& o) const { return std::tie(nss, any_of, sel, sels) < std::tie(o.nss, o.any_of, o.sel, o.sels); }
};

struct Ident {
  Str ns;
  Labels labels;
  bool deleting = false;
  bool operator<(const Ident& o) const { return std::tie(ns, labels, deleting) < std::tie(o.ns, o.labels, o.deleting); }
};

struct Term {  // ksim_aff_term
  int32_t kind, pair, gate, exist, self_ok;
  int64_t weight;
  bool operator<(const Term& o) const {
    return std::tie(kind, pair, gate, exist, self_ok, weight) < std::tie(o.kind, o.pair, o.gate, o.exist, o.self_ok, o.weight);
  }
};

struct AClass {
  std::vector<Term> req, pref;
  std::vector<std::pair<int32_t, int64_t>> carries;
  int32_t sp = -1;
  bool operator<(const AClass& o) const { return std::tie(req, pref, carries, sp) < std::tie(o.req, o.pref, o.carries, o.sp); }
};

struct AffinityIndex {
  std::vector<const Labels*> node_labels;
  int32_t hard_weight = 10;
  Interner<Str> keys;
  Interner<SelItem> sels;
  Interner<std::pair<int32_t, int32_t>> pairs;
  Interner<std::tuple<int32_t, int32_t, int32_t>> carry;
  Interner<Ident> idents;
  Interner<AClass> aclasses;

  AffinityIndex() {
    keys.get(Str("\x01" "all"));
    keys.get(Str("\x01" "node"));
  }

  std::pair<int32_t, Sel> sel_of(const PodObj& p, const PodTerm& t) {
    std::vector<Str> nss = t.nss;
    if (nss.empty()) nss.push_back(p.ns);
    std::sort(nss.begin(), nss.end());
    nss.erase(std::unique(nss.begin(), nss.end()), nss.end());
    Sel s;
    if (!from_label_selector(t.sel, &s)) fail(KSIM_E_UNSUPPORTED, "pod %s: affinity label selector does not parse", p.name.c_str());
    SelItem it;
    it.nss = nss;
    it.sel = s;
    return {sels.get(it), s};
  }

  int32_t ident(const PodObj& p) { return idents.get(Ident{p.ns, p.labels, p.deleting}); }

  static bool in(const std::vector<Str>& v, const Str& x) { return std::binary_search(v.begin(), v.end(), x); }

  static bool sel_matches(const Ident& id, const SelItem& s) {
    if (!in(s.nss, id.ns)) return false;
    if (s.any_of) {
      if (id.deleting) return false;
      for (const Sel& x : s.sels)
        if (matches(x, id.labels)) return true;
      return false;
    }
    return matches(s.sel, id.labels);
  }

  int32_t spread_pair(const PodObj& p) {
    if (p.spread.empty()) return -1;
    SelItem it;
    it.nss = {p.ns};
    it.any_of = true;
    it.sels = p.spread;
    const int32_t s = sels.get(it);
    keys.get(ZONE_KEY);
    return pairs.get({s, KEY_NODE});
  }

  int32_t aclass(const PodObj& p, bool with_spread) {
    const int32_t sp = with_spread ? spread_pair(p) : -1;
    if (!has_pod_affinity(p)) return sp < 0 ? -1 : aclasses.get(AClass{{}, {}, {}, sp});
    AClass ac;
    ac.sp = sp;
    const Ident me{p.ns, p.labels, p.deleting};
    for (int kind : {KSIM_AFF_REQ_AFFINITY, KSIM_AFF_REQ_ANTI}) {
      const std::vector<PodTerm>& ts = kind == KSIM_AFF_REQ_AFFINITY ? p.a_req : p.n_req;
      for (const PodTerm& t : ts) {
        if (t.key.empty()) fail(KSIM_E_UNSUPPORTED, "pod %s: required pod (anti-)affinity term without topologyKey", p.name.c_str());
        const int32_t s = sel_of(p, t).first;
        int32_t mp, gate, ep;
        if (t.key == HOSTNAME) {
          mp = pairs.get({s, KEY_NODE});
          gate = keys.get(t.key);
          ep = mp;
        } else {
          const int32_t k = keys.get(t.key);
          mp = pairs.get({s, k});
          gate = k;
          ep = pairs.get({s, KEY_ALL});
        }
        const int32_t self_ok = sel_matches(me, sels.items[s]) ? 1 : 0;
        ac.req.push_back(Term{kind, mp, gate, ep, self_ok, 0});
      }
    }
    for (int sign : {1, -1}) {
      if (sign > 0 ? !p.has_pa : !p.has_anti) continue;
      for (const PodTerm& t : sign > 0 ? p.a_pref : p.n_pref) {
        const auto sv = sel_of(p, t);
        if (t.key.empty() || sv.second.nothing) continue;
        ac.pref.push_back(Term{KSIM_AFF_PREFERRED, pairs.get({sv.first, keys.get(t.key)}), 0, 0, 0, (int64_t)sign * t.weight});
      }
    }
    std::map<int32_t, int64_t> carries;
    auto add_carry = [&](const PodTerm& t, int32_t kind, int64_t amount) {
      const auto sv = sel_of(p, t);
      if (t.key.empty()) {
        if (kind == KSIM_AFF_CARRY_ANTI) fail(KSIM_E_UNSUPPORTED, "pod %s: required anti-affinity term without topologyKey", p.name.c_str());
        return;
      }
      if (sv.second.nothing) return;
      const int32_t e = carry.get(std::make_tuple(sv.first, keys.get(t.key), kind));
      carries[e] += amount;
    };
    for (const PodTerm& t : p.n_req) add_carry(t, KSIM_AFF_CARRY_ANTI, 1);
    if (p.has_pa) {
      if (hard_weight > 0)
        for (const PodTerm& t : p.a_req) add_carry(t, KSIM_AFF_CARRY_PRIO, hard_weight);
      for (const PodTerm& t : p.a_pref) add_carry(t, KSIM_AFF_CARRY_PRIO, t.weight);
    }
    if (p.has_anti)
      for (const PodTerm& t : p.n_pref) add_carry(t, KSIM_AFF_CARRY_PRIO, -(int64_t)t.weight);
    for (const auto& e : carries)
      if (e.second != 0 || std::get<2>(carry.items[e.first]) == KSIM_AFF_CARRY_ANTI) ac.carries.push_back(e);
    std::stable_sort(ac.req.begin(), ac.req.end(),
                     [](const Term& a, const Term& b) { return (a.kind != KSIM_AFF_REQ_AFFINITY) < (b.kind != KSIM_AFF_REQ_AFFINITY); });
    if (ac.req.empty() && ac.pref.empty() && ac.carries.empty() && sp < 0) return -1;
    return aclasses.get(ac);
  }
};

struct AffTables {
  int32_t n_keys = 0, n_sel = 0, n_ident = 0, n_pair = 0, n_carry = 0, n_aclass = 0, sw = 0, cw = 0, zone_key = -1;
  std::vector<int32_t> dom, n_dom, pair_sel, pair_key, carry_key, carry_kind, ac, spread_pair, cnt;
  std::vector<int64_t> pair_off, carry_off, carried;
  std::vector<uint64_t> isel, ianti, iprio;
  std::vector<ksim_aff_term> terms;
  std::vector<ksim_aff_carry> carries;
  std::vector<int32_t> remap;  // interned identity -> aff_ident
};

// ---------------------------------------------------------------- volumes (volumes.py)
struct VolKey {
  Str tag, a, b, c;
  bool operator<(const VolKey& o) const { return std::tie(tag, a, b, c) < std::tie(o.tag, o.a, o.b, o.c); }
};

struct ZoneEntry {  // one PVC's VolumeZone input: error / skip / the PV's zone labels
  int kind = 0;     // 0 labels, 1 error, 2 skip
  std::vector<std::pair<Str, Str>> labels;
  bool operator<(const ZoneEntry& o) const { return std::tie(kind, labels) < std::tie(o.kind, o.labels); }
};

struct PV {
  Labels labels;
  int32_t kind = 0;
  Str id;
  bool node_affinity = false;
};
struct PVC {
  Str volume_name;
  bool has_sc = false;
  Str sc;
};

const uint32_t ALL_FILTERS = KSIM_VOL_EBS | KSIM_VOL_GCE_PD | KSIM_VOL_AZURE_DISK;
const char* const ZONE_LABEL = "failure-domain.beta.kubernetes.io/zone";
const char* const REGION_LABEL = "failure-domain.beta.kubernetes.io/region";

struct VolumeIndex {
  std::map<Str, PV> pvs;
  std::map<std::pair<Str, Str>, PVC> pvcs;
  std::map<Str, std::pair<bool, Str>> scs;  // name -> (binding mode set, mode)
  Interner<VolKey> keys;
  std::vector<uint32_t> key_filter;
  std::map<std::pair<std::vector<std::pair<int32_t, uint32_t>>, std::vector<ZoneEntry>>, int32_t> classes;
  std::vector<std::vector<std::pair<int32_t, uint32_t>>> class_refs;
  std::vector<uint32_t> class_filter;
  std::vector<std::vector<ZoneEntry>> class_zone;
  bool err_claim = false, err_binding = false;

  int32_t key(const VolKey& k, uint32_t filt) {
    const int32_t n = (int32_t)keys.items.size();
    const int32_t i = keys.get(k);
    if (i == n) key_filter.push_back(filt);
    return i;
  }

  // the PV behind a PVC as MaxPD resolves it; false when the PV is not of a counted kind
  bool pvc_target(const Str& ns, const Str& claim, VolKey* k, uint32_t* f) {
    auto pc = pvcs.find({ns, claim});
    const PV* pv = nullptr;
    if (pc != pvcs.end() && !pc->second.volume_name.empty()) {
      auto it = pvs.find(pc->second.volume_name);
      if (it != pvs.end()) pv = &it->second;
    }
    if (!pv) {
      *k = VolKey{"PVC", ns, claim, ""};
      *f = ALL_FILTERS;
      return true;
    }
    switch (pv->kind) {
      case KSIM_K8S_VOL_EBS: *k = VolKey{"EBS", pv->id, "", ""}; *f = KSIM_VOL_EBS; return true;
      case KSIM_K8S_VOL_GCE_PD: *k = VolKey{"GCE", pv->id, "", ""}; *f = KSIM_VOL_GCE_PD; return true;
      case KSIM_K8S_VOL_AZURE_DISK: *k = VolKey{"AZ", pv->id, "", ""}; *f = KSIM_VOL_AZURE_DISK; return true;
      default: return false;
    }
  }

  ZoneEntry zone_entry(const Str& ns, const Str& claim) {
    ZoneEntry z;
    auto pc = pvcs.find({ns, claim});
    if (pc == pvcs.end()) { z.kind = 1; return z; }
    if (pc->second.volume_name.empty()) {
      if (pc->second.has_sc && !pc->second.sc.empty()) {
        auto s = scs.find(pc->second.sc);
        if (s != scs.end()) {
          if (!s->second.first) { z.kind = 1; return z; }
          if (s->second.second == "WaitForFirstConsumer") { z.kind = 2; return z; }
        }
      }
      z.kind = 1;
      return z;
    }
    auto it = pvs.find(pc->second.volume_name);
    if (it == pvs.end()) { z.kind = 1; return z; }
    for (const auto& l : it->second.labels)
      if (l.first == ZONE_LABEL || l.first == REGION_LABEL) z.labels.push_back(l);
    return z;
  }

  void binding_check(const Str& ns, const Str& claim) {
    auto pc = pvcs.find({ns, claim});
    const PV* pv = nullptr;
    if (pc != pvcs.end()) {
      auto it = pvs.find(pc->second.volume_name);
      if (it != pvs.end()) pv = &it->second;
    }
    if (!pv || pv->node_affinity) err_binding = true;
  }

  // (refs, zone list, has a PVC) of one pod's volumes
  void refs(const PodObj& p, bool queued, std::vector<std::pair<int32_t, uint32_t>>* out, std::vector<ZoneEntry>* zone,
            bool* has_pvc) {
    *has_pvc = false;
    for (const Volume& v : p.vols) {
      const uint32_t ro_rw = KSIM_VOL_CONFLICT_RW | KSIM_VOL_READ_ONLY;
      switch (v.kind) {
        case KSIM_K8S_VOL_GCE_PD:
          out->push_back({key(VolKey{"GCE", v.id, "", ""}, KSIM_VOL_GCE_PD), v.ro ? ro_rw : KSIM_VOL_CONFLICT_ANY});
          break;
        case KSIM_K8S_VOL_EBS:
          out->push_back({key(VolKey{"EBS", v.id, "", ""}, KSIM_VOL_EBS), KSIM_VOL_CONFLICT_ANY | (v.ro ? KSIM_VOL_READ_ONLY : 0u)});
          break;
        case KSIM_K8S_VOL_ISCSI:
          out->push_back({key(VolKey{"ISCSI", v.id, "", ""}, 0), v.ro ? ro_rw : KSIM_VOL_CONFLICT_ANY});
          break;
        case KSIM_K8S_VOL_RBD: {
          std::vector<Str> seen;
          for (const Str& m : v.monitors) {  // haveOverlap: some monitor shared
            if (std::find(seen.begin(), seen.end(), m) != seen.end()) continue;
            seen.push_back(m);
            out->push_back({key(VolKey{"RBD", m, v.pool, v.image}, 0), v.ro ? ro_rw : KSIM_VOL_CONFLICT_ANY});
          }
          break;
        }
        case KSIM_K8S_VOL_AZURE_DISK:
          out->push_back({key(VolKey{"AZ", v.id, "", ""}, KSIM_VOL_AZURE_DISK), 0u});
          break;
        case KSIM_K8S_VOL_PVC: {
          *has_pvc = true;
          if (v.id.empty()) {
            err_claim = true;
            ZoneEntry e;
            e.kind = 1;
            zone->push_back(e);
            continue;
          }
          VolKey k;
          uint32_t f;
          if (pvc_target(p.ns, v.id, &k, &f)) out->push_back({key(k, f), KSIM_VOL_VIA_PVC});
          if (queued) {
            zone->push_back(zone_entry(p.ns, v.id));
            binding_check(p.ns, v.id);
          }
          break;
        }
        default:
          break;
      }
    }
  }

  int32_t vclass(const PodObj& p) {
    std::vector<std::pair<int32_t, uint32_t>> refs_;
    std::vector<ZoneEntry> zone;
    bool has_pvc;
    refs(p, true, &refs_, &zone, &has_pvc);
    if (refs_.empty() && !has_pvc) return 0;
    std::set<int32_t> seen;
    uint32_t filt = 0;
    std::vector<std::pair<int32_t, uint32_t>> flagged;
    for (auto r : refs_) {
      const uint32_t kf = key_filter[r.first];
      if (kf && !seen.count(r.first)) r.second |= KSIM_VOL_NEW;
      seen.insert(r.first);
      filt |= kf;
      flagged.push_back(r);
    }
    auto k = std::make_pair(flagged, zone);
    auto it = classes.find(k);
    if (it != classes.end()) return it->second + 1;
    const int32_t c = (int32_t)class_refs.size();
    classes.emplace(k, c);
    class_refs.push_back(flagged);
    class_filter.push_back(filt);
    class_zone.push_back(zone);
    return c + 1;
  }
};

// volumeutil.LabelZonesToSet; false on a parse error
bool zones_of(const Str& v, std::set<Str>* out) {
  size_t i = 0;
  for (;;) {
    const size_t j = v.find("__", i);
    Str t = v.substr(i, j == Str::npos ? Str::npos : j - i);
    const size_t a = t.find_first_not_of(" \t\n\r\f\v"), b = t.find_last_not_of(" \t\n\r\f\v");
    t = a == Str::npos ? Str() : t.substr(a, b - a + 1);
    if (t.empty()) return false;
    out->insert(t);
    if (j == Str::npos) return true;
    i = j + 2;
  }
}


// ---------------------------------------------------------------- node objects
constexpr int64_t MIN_IMG_SIZE = 23ll * 1024 * 1024, MAX_IMG_SIZE = 1000ll * 1024 * 1024;  // image_locality.go:29-33

// calculateScoreFromSize over totalImageSize (image_locality.go:39-88): the summed sizes of the pod's
// container images the node lists, bucketed 0..10.
int64_t image_score(const std::vector<Str>& pod_images, const std::vector<std::pair<Str, int64_t>>& node_images) {
  int64_t total = 0;
  for (const Str& i : pod_images) {
    auto it = std::lower_bound(node_images.begin(), node_images.end(), std::make_pair(i, INT64_MIN));
    if (it != node_images.end() && it->first == i) total += it->second;
  }
  if (total == 0 || total < MIN_IMG_SIZE) return 0;
  if (total >= MAX_IMG_SIZE) return 10;
  return 10 * (total - MIN_IMG_SIZE) / (MAX_IMG_SIZE - MIN_IMG_SIZE) + 1;
}

NodeObj copy_node(const ksim_k8s_node& x) {
  NodeObj o;
  o.name = S(x.name);
  for (int32_t i = 0; i < x.n_labels; ++i) o.labels[S(x.labels[i].key)] = S(x.labels[i].value);
  for (int32_t i = 0; i < x.n_taints; ++i) o.taints.push_back(Taint{S(x.taints[i].key), S(x.taints[i].value), S(x.taints[i].effect)});
  o.unschedulable = x.unschedulable != 0;
  for (int32_t i = 0; i < x.n_conditions; ++i) o.conds.push_back({S(x.conditions[i].type), S(x.conditions[i].status)});
  o.alloc[0] = x.alloc_cpu_milli; o.alloc[1] = x.alloc_mem; o.alloc[2] = x.alloc_gpu; o.alloc[3] = x.alloc_eph;
  o.pods = x.alloc_pods;
  for (int32_t i = 0; i < x.n_alloc_other; ++i) o.other.push_back({S(x.alloc_other[i].name), x.alloc_other[i].value});
  for (int32_t i = 0; i < x.n_avoid; ++i) o.avoid.push_back(Avoid{x.avoid[i].has_controller != 0, S(x.avoid[i].kind), S(x.avoid[i].uid)});
  std::map<Str, int64_t> imgs;  // totalImageSize: every name of every image; a later image's size wins
  for (int32_t i = 0; i < x.n_images; ++i)
    for (int32_t k = 0; k < x.images[i].n_names; ++k) imgs[S(x.images[i].names[k])] = x.images[i].size_bytes;
  o.images.assign(imgs.begin(), imgs.end());
  o.has_images = x.has_images != 0 || x.n_images > 0;
  return o;
}

// NodeInfo.SetNode + CheckNodeConditionPredicate's condition bits (ingest.node_static).  SetNode keeps
// the last MemoryPressure / DiskPressure condition's status and leaves the previous one when the node
// has none (mem / disk: the previous status in, "" = none; the new one out).
uint32_t node_flags(const NodeObj& x, Str* mem = nullptr, Str* disk = nullptr) {
  uint32_t f = 0;
  Str m = mem ? *mem : Str(), d = disk ? *disk : Str();
  bool seen[3] = {false, false, false};
  for (const auto& cd : x.conds) {
    const Str& t = cd.first;
    const Str& st = cd.second;
    int b = -1;
    if (t == "Ready" && st != "True") b = 0;
    else if (t == "OutOfDisk" && st != "False") b = 1;
    else if (t == "NetworkUnavailable" && st != "False") b = 2;
    if (b >= 0) {
      if (seen[b]) fail(KSIM_E_UNSUPPORTED, "node %s: repeated failing %s condition", x.name.c_str(), t.c_str());
      seen[b] = true;
      f |= b == 0 ? KSIM_N_NOT_READY : b == 1 ? KSIM_N_OUT_OF_DISK : KSIM_N_NET_UNAVAIL;
    }
    if (t == "MemoryPressure") m = st;
    else if (t == "DiskPressure") d = st;
  }
  if (m == "True") f |= KSIM_N_MEM_PRESSURE;
  if (d == "True") f |= KSIM_N_DISK_PRESSURE;
  if (x.unschedulable) f |= KSIM_N_UNSCHEDULABLE;
  if (mem) *mem = m;
  if (disk) *disk = d;
  return f;
}

// CalculateNodePreferAvoidPodsPriorityMap for a pod whose RC / RS controllerRef is (kind, uid).
int64_t avoid_score(const std::vector<Avoid>& entries, const Str& kind, const Str& uid) {
  for (const Avoid& e : entries) {
    if (!e.has) fail(KSIM_E_UNSUPPORTED, "preferAvoidPods entry without a podController (the reference dereferences nil)");
    if (e.kind == kind && e.uid == uid) return 0;
  }
  return 10;
}

uint64_t port_key(int32_t ip, int32_t proto, int32_t port) { return KSIM_PORT_KEY(ip, proto, port); }

// Runs f, turning a Fail (or any exception) into a status code and the owner's error text.
template <class Owner>
int guard(Owner* o, const std::function<void()>& f) {
  try {
    f();
    return KSIM_OK;
  } catch (const Fail& e) {
    if (o) o->err = e.msg;
    return e.code;
  } catch (const std::exception& e) {
    if (o) o->err = e.what();
    return KSIM_E_INVAL;
  }
}

// ---------------------------------------------------------------- interned inputs and class tables
struct Interns {
  Interner<LabelSetKey> label_sets;
  Interner<std::vector<Taint>> taint_sets;
  Interner<Str> scalar_names, ips, protos;
  Interner<ClassKey> classes;
  bool images = false;  // ImageLocality's inputs interned: node images in label sets, pod images in classes
  Interns() {
    ips.get("0.0.0.0");  // id 0 = wildcard
    protos.get("TCP");   // id 0 = default protocol
  }
  int32_t label_set(const NodeObj& x) { return label_sets.get(LabelSetKey{x.labels, x.avoid, images ? x.images : decltype(x.images){}}); }
};

// Per (pod class x label set / taint set): podMatchesNodeLabels, PodToleratesNodeTaints (NoSchedule +
// NoExecute; NoExecute only), the TaintToleration / NodeAffinity map values as reduce classes, and the
// raw inputs of the NodeAffinity class dimension's addends (preferred weight, NodePreferAvoidPods and
// ImageLocality map scores) — ingest.build_class_tables.
struct ClassTab {
  int32_t Cn = 0, L = 0, T = 0, lw = 0, tw = 0;
  int32_t val_w = KSIM_MAX_RCLASS;  // row width of tt_val / na_val (ksim_class_tables.val_width)
  std::vector<uint32_t> sel_ok, taint_ok, noexec_ok;
  std::vector<uint8_t> tt_class, na_class;
  std::vector<int32_t> n_tt, n_na;
  std::vector<int64_t> tt_val, na_val, na_w, na_p, im_s;
  std::vector<uint32_t> need;  // KSIM_POD_NEED_* per class
  std::set<int32_t> bad_classes;  // a preferred node-affinity term does not parse
  bool pa_split = false, im_any = false;
};

void build_class_tab(const Interns& in, ClassTab* c) {
  const int32_t L = (int32_t)in.label_sets.items.size(), T = (int32_t)in.taint_sets.items.size();
  const int32_t Cn = std::max<int32_t>((int32_t)in.classes.items.size(), 1);
  const int32_t lw = (L + 31) / 32, tw = (T + 31) / 32;
  c->Cn = Cn; c->L = L; c->T = T; c->lw = lw; c->tw = tw;
  c->sel_ok.assign((size_t)Cn * lw, 0);
  c->taint_ok.assign((size_t)Cn * tw, 0);
  c->noexec_ok.assign((size_t)Cn * tw, 0);
  c->tt_class.assign((size_t)Cn * T, 0);
  c->na_class.assign((size_t)Cn * L, 0);
  c->n_tt.assign(Cn, 1);
  c->n_na.assign(Cn, 1);
  c->na_w.assign((size_t)Cn * L, 0);
  c->na_p.assign((size_t)Cn * L, 10);
  c->im_s.assign((size_t)Cn * L, 0);
  c->need.assign(Cn, 0);
  c->bad_classes.clear();
  c->pa_split = false;
  c->im_any = false;
  std::vector<std::vector<int64_t>> tvs(Cn), avs(Cn);  // per class: its distinct values (rows written below)
  for (int32_t k = 0; k < Cn; ++k) {
    const bool real = k < (int32_t)in.classes.items.size();
    const PodObj spec = real ? class_pod(in.classes.items[k]) : PodObj{};
    const std::vector<Str> no_images;
    const std::vector<Str>& imgs = real ? in.classes.items[k].images : no_images;
    std::vector<Tol> prefer;
    for (const Tol& t : spec.tols)
      if (t.effect.empty() || t.effect == "PreferNoSchedule") prefer.push_back(t);
    bool all_sel = true, all_taint = true;
    std::vector<int64_t> weights, pas, counts;
    for (int32_t li = 0; li < L; ++li) {
      const LabelSetKey& ls = in.label_sets.items[li];
      pas.push_back(spec.has_ctrl ? avoid_score(ls.avoid, spec.ctrl_kind, spec.ctrl_uid) : 10);
      if (!imgs.empty()) {
        c->im_s[(size_t)k * L + li] = image_score(imgs, ls.images);
        c->im_any |= c->im_s[(size_t)k * L + li] != 0;
      }
      const bool ok = pod_matches_node_labels(spec, ls.labels);
      if (ok) c->sel_ok[(size_t)k * lw + (li >> 5)] |= 1u << (li & 31);
      all_sel &= ok;
      int64_t w = 0;
      if (!preferred_weight(spec, ls.labels, &w)) {
        c->bad_classes.insert(k);
        w = 0;
      }
      weights.push_back(w);
    }
    for (int32_t ti = 0; ti < T; ++ti) {
      const std::vector<Taint>& ts = in.taint_sets.items[ti];
      auto tolerated = [&](const Taint& x, const std::vector<Tol>& tols) {
        for (const Tol& t : tols)
          if (tolerates(t, x)) return true;
        return false;
      };
      bool ok = true, ok2 = true;
      int64_t cnt = 0;
      for (const Taint& x : ts) {
        if ((x.effect == "NoSchedule" || x.effect == "NoExecute") && !tolerated(x, spec.tols)) ok = false;
        if (x.effect == "NoExecute" && !tolerated(x, spec.tols)) ok2 = false;
        if (x.effect == "PreferNoSchedule" && !tolerated(x, prefer)) ++cnt;
      }
      if (ok) c->taint_ok[(size_t)k * tw + (ti >> 5)] |= 1u << (ti & 31);
      if (ok2) c->noexec_ok[(size_t)k * tw + (ti >> 5)] |= 1u << (ti & 31);
      all_taint &= ok && ok2;
      counts.push_back(cnt);
    }
    std::vector<int64_t> tv(counts), av(weights);
    std::sort(tv.begin(), tv.end()); tv.erase(std::unique(tv.begin(), tv.end()), tv.end());
    std::sort(av.begin(), av.end()); av.erase(std::unique(av.begin(), av.end()), av.end());
    if (tv.empty()) tv.push_back(0);  // an empty taint-set list still has one class
    if (av.empty()) av.push_back(0);
    // NormalizeReduce takes any number of values (reduce.go:29-64); the reduce classes of one pod
    // are bounded by the launch form's wide decision (a product above 16 decides there)
    if (tv.size() * av.size() > KSIM_MAX_WIDE)
      fail(KSIM_E_UNSUPPORTED, "pod class needs %zu x %zu reduce classes (> %d)", tv.size(), av.size(), KSIM_MAX_WIDE);
    c->n_tt[k] = (int32_t)tv.size();
    c->n_na[k] = (int32_t)av.size();
    for (int32_t ti = 0; ti < T; ++ti)
      c->tt_class[(size_t)k * T + ti] = (uint8_t)(std::lower_bound(tv.begin(), tv.end(), counts[ti]) - tv.begin());
    for (int32_t li = 0; li < L; ++li) {
      c->na_class[(size_t)k * L + li] = (uint8_t)(std::lower_bound(av.begin(), av.end(), weights[li]) - av.begin());
      c->na_w[(size_t)k * L + li] = weights[li];
      c->na_p[(size_t)k * L + li] = pas[li];
    }
    for (int32_t li = 1; li < L; ++li) c->pa_split |= pas[li] != pas[0];
    c->need[k] = (all_sel ? 0u : KSIM_POD_NEED_SELECTOR) | (all_taint ? 0u : KSIM_POD_NEED_TAINTS);
    tvs[k] = std::move(tv);
    avs[k] = std::move(av);
  }
  int32_t W = KSIM_MAX_RCLASS;
  for (int32_t k = 0; k < Cn; ++k) W = std::max<int32_t>(W, (int32_t)std::max(tvs[k].size(), avs[k].size()));
  c->val_w = W;
  c->tt_val.assign((size_t)Cn * W, 0);
  c->na_val.assign((size_t)Cn * W, 0);
  for (int32_t k = 0; k < Cn; ++k) {
    for (size_t q = 0; q < tvs[k].size(); ++q) c->tt_val[(size_t)k * W + q] = tvs[k][q];
    for (size_t q = 0; q < avs[k].size(); ++q) c->na_val[(size_t)k * W + q] = avs[k][q];
  }
}

// A Policy's arguments over the interned label sets and classes (scheduler.plan's
// label_presence_flags, service_affinity_table and label_set_priority, restated).
struct PolicyArgs {
  bool on = false;
  std::vector<Str> presence_labels;
  bool presence = true;
  std::vector<Str> affinity_labels;
  std::vector<std::pair<Str, std::pair<bool, int64_t>>> label_prios;  // label -> (presence, weight)
};

// CheckNodeLabelPresence (predicates.go:875-910): per label set, whether it fails.
std::vector<uint8_t> policy_presence_bad(const Interns& in, const PolicyArgs& a) {
  std::vector<uint8_t> bad(in.label_sets.items.size(), 0);
  for (size_t li = 0; li < bad.size(); ++li)
    for (const Str& l : a.presence_labels)
      if ((in.label_sets.items[li].labels.count(l) != 0) != a.presence) { bad[li] = 1; break; }
  return bad;
}

// labelPreference (node_label.go:42-58): per label set, the weighted MaxPriority sum.
std::vector<int64_t> policy_label_add(const Interns& in, const PolicyArgs& a) {
  std::vector<int64_t> add(in.label_sets.items.size(), 0);
  for (size_t li = 0; li < add.size(); ++li)
    for (const auto& pr : a.label_prios)
      if ((in.label_sets.items[li].labels.count(pr.first) != 0) == pr.second.first) add[li] += 10 * pr.second.second;
  return add;
}

// CheckServiceAffinity with no service selecting the pod (predicates.go:980-1016): per (class, label
// set) the class's nodeSelector values of the listed labels must be the node's (FindLabelsInSet,
// CreateSelectorFromLabels); need[class] when it fails somewhere.
void policy_svc_ok(const Interns& in, const ClassTab& ct, const PolicyArgs& a, std::vector<uint32_t>* ok,
                   std::vector<uint8_t>* need) {
  const int32_t Cn = ct.Cn, L = ct.L, lw = std::max<int32_t>((L + 31) / 32, 1);
  ok->assign((size_t)Cn * lw, 0);
  need->assign(Cn, 0);
  for (int32_t k = 0; k < Cn; ++k) {
    std::vector<std::pair<Str, Str>> al;
    if (k < (int32_t)in.classes.items.size())
      for (const auto& kv : in.classes.items[k].ns)
        if (std::find(a.affinity_labels.begin(), a.affinity_labels.end(), kv.first) != a.affinity_labels.end())
          al.push_back(kv);
    for (int32_t li = 0; li < L; ++li) {
      const Labels& lab = in.label_sets.items[li].labels;
      bool m = true;
      for (const auto& kv : al) {
        auto it = lab.find(kv.first);
        if (it == lab.end() || it->second != kv.second) { m = false; break; }
      }
      if (m) (*ok)[(size_t)k * lw + (li >> 5)] |= 1u << (li & 31);
      else (*need)[k] = 1;
    }
  }
}

// scheduler.class_tables_for: NodePreferAvoidPods' and ImageLocality's weighted map scores as
// per-class addends when the policy weighs them and they tell some class's nodes apart — the
// NodeAffinity class dimension re-keyed by (preferred weight, summed addend).  Returns whether the
// addends apply; *pa_on: NodePreferAvoidPods rides them (its constant leaves const_score).
// *val_w: the row width of nav / add (the class table's, or wider when an addend splits more classes).
bool class_addends(const ClassTab& c, int64_t w_pa, int64_t w_im, bool use_w, std::vector<uint8_t>* nac,
                   std::vector<int32_t>* nna, std::vector<int64_t>* nav, std::vector<int64_t>* add, bool* pa_on_out,
                   const std::vector<int64_t>* lab_add = nullptr, int32_t* val_w = nullptr) {
  const bool pa_on = w_pa && c.pa_split, im_on = w_im && c.im_any;
  bool lab_on = false;  // a Policy's label priorities (per label set, weighted)
  if (lab_add)
    for (int64_t v : *lab_add) lab_on |= v != 0;
  if (pa_on_out) *pa_on_out = pa_on;
  if (!pa_on && !im_on && !lab_on) return false;
  const int32_t Cn = c.Cn, L = c.L;
  nac->assign((size_t)Cn * L, 0);
  nna->assign(Cn, 1);
  std::vector<std::vector<std::pair<int64_t, int64_t>>> avs(Cn);
  for (int32_t k = 0; k < Cn; ++k) {
    std::vector<std::pair<int64_t, int64_t>> keys;
    for (int32_t li = 0; li < L; ++li) {
      const size_t x = (size_t)k * L + li;
      keys.push_back({use_w ? c.na_w[x] : 0, (pa_on ? c.na_p[x] * w_pa : 0) + (im_on ? c.im_s[x] * w_im : 0) +
                                                 (lab_on ? (*lab_add)[li] : 0)});
    }
    std::vector<std::pair<int64_t, int64_t>> av(keys);
    std::sort(av.begin(), av.end());
    av.erase(std::unique(av.begin(), av.end()), av.end());
    if ((size_t)c.n_tt[k] * av.size() > KSIM_MAX_WIDE)
      fail(KSIM_E_UNSUPPORTED, "pod class needs %d x %zu reduce classes (> %d)", c.n_tt[k], av.size(), KSIM_MAX_WIDE);
    (*nna)[k] = (int32_t)av.size();
    for (int32_t li = 0; li < L; ++li)
      (*nac)[(size_t)k * L + li] = (uint8_t)(std::lower_bound(av.begin(), av.end(), keys[li]) - av.begin());
    avs[k] = std::move(av);
  }
  int32_t W = c.val_w;
  for (int32_t k = 0; k < Cn; ++k) W = std::max<int32_t>(W, (int32_t)avs[k].size());
  nav->assign((size_t)Cn * W, 0);
  add->assign((size_t)Cn * W, 0);
  for (int32_t k = 0; k < Cn; ++k)
    for (size_t q = 0; q < avs[k].size(); ++q) {
      (*nav)[(size_t)k * W + q] = avs[k][q].first;
      (*add)[(size_t)k * W + q] = avs[k][q].second;
    }
  if (val_w) *val_w = W;
  return true;
}

// tt_val rows of width c.val_w re-laid out at width w (>= c.val_w).
std::vector<int64_t> widen_rows(const std::vector<int64_t>& v, int32_t Cn, int32_t from, int32_t w) {
  std::vector<int64_t> o((size_t)Cn * w, 0);
  for (int32_t k = 0; k < Cn; ++k)
    for (int32_t q = 0; q < from; ++q) o[(size_t)k * w + q] = v[(size_t)k * from + q];
  return o;
}

// ksim_load_classes over a ClassTab (with the addends of class_addends when they apply).
int load_class_tab(const ClassTab& c, ksim_handle* h, int64_t w_pa, int64_t w_im, bool use_w, const uint32_t* svc_ok = nullptr,
                   const std::vector<int64_t>* lab_add = nullptr) {
  std::vector<uint8_t> nac;
  std::vector<int32_t> nna;
  std::vector<int64_t> nav, add;
  int32_t W = c.val_w;
  const bool pa = class_addends(c, w_pa, w_im, use_w, &nac, &nna, &nav, &add, nullptr, lab_add, &W);
  // one row width for every value array (the addends may have split more NodeAffinity classes)
  const std::vector<int64_t> ttw = W > c.val_w ? widen_rows(c.tt_val, c.Cn, c.val_w, W) : std::vector<int64_t>();
  ksim_class_tables t{};
  t.val_width = W;
  t.n_classes = c.Cn;
  t.n_label_sets = c.L;
  t.n_taint_sets = c.T;
  t.sel_ok = c.sel_ok.data();
  t.taint_ok = c.taint_ok.data();
  t.noexec_ok = c.noexec_ok.data();
  t.tt_class = c.tt_class.data();
  t.na_class = pa ? nac.data() : c.na_class.data();
  t.n_tt = c.n_tt.data();
  t.n_na = pa ? nna.data() : c.n_na.data();
  t.tt_val = W > c.val_w ? ttw.data() : c.tt_val.data();
  t.na_val = pa ? nav.data() : c.na_val.data();
  t.na_add = pa ? add.data() : nullptr;
  t.svc_ok = svc_ok;
  return ksim_load_classes(h, &t);
}

// One pod → its descriptor (ingest.Cluster.encode_pod): requests, flags, spec.nodeName's rank in
// `index` (-2 when it names no listed node), its class (interned), its host-port keys and scalar
// requests appended to `ports` / `scalars` (port_off / scalar_off index them).  Affinity / volume
// ids are left 0.
void encode_pod_row(Interns& in, const std::map<Str, int64_t>& index, const PodObj& p, const Compiled& cr, ksim_pod* row,
                    std::vector<uint64_t>* ports, std::vector<ksim_scalar_req>* scalars) {
  memset(row, 0, sizeof *row);
  row->req_cpu = cr.pred.cpu; row->req_mem = cr.pred.mem; row->req_gpu = cr.pred.gpu; row->req_eph = cr.pred.eph;
  row->add_cpu = cr.add.cpu; row->add_mem = cr.add.mem; row->add_gpu = cr.add.gpu; row->add_eph = cr.add.eph;
  row->nz_cpu = cr.nzc; row->nz_mem = cr.nzm;
  uint32_t fl = 0;
  if (cr.pred.cpu || cr.pred.mem || cr.pred.gpu || cr.pred.eph || !cr.pred.scalar.empty()) fl |= KSIM_POD_ANY_REQUEST;
  if (best_effort(p)) fl |= KSIM_POD_BEST_EFFORT;
  if (p.node_name.empty()) row->host = -1;
  else {
    auto it = index.find(p.node_name);
    row->host = it == index.end() ? -2 : (int32_t)it->second;
  }
  row->cls = in.classes.get(class_key(p, in.images));
  row->flags = fl;
  const auto hp = host_ports(p);
  row->port_off = (int32_t)ports->size();
  row->port_cnt = (int32_t)hp.size();
  for (const auto& e : hp) ports->push_back(port_key(in.ips.get(std::get<0>(e)), in.protos.get(std::get<1>(e)), std::get<2>(e)));
  row->scalar_off = (int32_t)scalars->size();
  row->scalar_cnt = (int32_t)cr.pred.scalar.size();
  Res add = cr.add;
  for (const auto& e : cr.pred.scalar) {
    const int32_t col = in.scalar_names.find(e.first);
    if (col < 0) fail(KSIM_E_UNSUPPORTED, "pod %s: scalar resource %s is not a column of the node table", p.name.c_str(), e.first.c_str());
    const int64_t* a = add.find(e.first);
    scalars->push_back(ksim_scalar_req{col, 0, e.second, a ? *a : 0});
  }
}

// ---------------------------------------------------------------- affinity tables (affinity.py build)
struct Placed {  // a pod cached on a listed node, as the affinity tables count it
  int64_t node;
  int32_t ident, aclass;
};

// The affinity tables from an index and the placed pods; keep_all: every interned identity keeps an
// id (1 + index) instead of dropping the ones that match nothing.
void build_aff_tables(const AffinityIndex& idx, const std::vector<const Labels*>& node_labels, const std::vector<Placed>& placed,
                      bool keep_all, AffTables* out) {
  if (idx.sels.items.size() > KSIM_AFF_MAX_SEL) fail(KSIM_E_UNSUPPORTED, "more than %d distinct inter-pod affinity selectors", KSIM_AFF_MAX_SEL);
  if (idx.carry.items.size() > KSIM_AFF_MAX_CARRY) fail(KSIM_E_UNSUPPORTED, "more than %d distinct carried inter-pod affinity terms", KSIM_AFF_MAX_CARRY);
  AffTables& t = *out;
  t = AffTables();
  const int64_t n = (int64_t)node_labels.size();
  const int32_t K = (int32_t)idx.keys.items.size();
  t.n_keys = K;
  t.dom.assign((size_t)K * n, -1);
  t.n_dom.assign(K, 0);
  for (int64_t i = 0; i < n; ++i) { t.dom[KEY_ALL * n + i] = 0; t.dom[KEY_NODE * n + i] = (int32_t)i; }
  t.n_dom[KEY_ALL] = 1;
  t.n_dom[KEY_NODE] = (int32_t)n;
  for (int32_t k = 2; k < K; ++k) {
    const Str& name = idx.keys.items[k];
    std::map<Str, int32_t> vals;
    for (int64_t i = 0; i < n; ++i) {
      const Labels& lab = *node_labels[i];
      Str v;
      if (name == ZONE_KEY) {
        v = zone_key_of(lab);
        if (v.empty()) continue;
      } else {
        auto it = lab.find(name);
        if (it == lab.end()) continue;
        v = it->second;
      }
      auto ins = vals.emplace(v, (int32_t)vals.size());
      t.dom[(size_t)k * n + i] = ins.first->second;
    }
    t.n_dom[k] = (int32_t)vals.size();
  }
  const int32_t I = (int32_t)idx.idents.items.size(), NS = (int32_t)idx.sels.items.size();
  const int32_t E = (int32_t)idx.carry.items.size(), P = (int32_t)idx.pairs.items.size();
  const int32_t SW = (NS + 63) / 64, CW = (E + 63) / 64;
  std::vector<uint64_t> isel((size_t)I * SW, 0), ianti((size_t)I * CW, 0), iprio((size_t)I * CW, 0);
  std::vector<uint8_t> live(I, 0);
  for (int32_t i = 0; i < I; ++i) {
    std::vector<uint8_t> hit(NS, 0);
    for (int32_t s = 0; s < NS; ++s) {
      hit[s] = AffinityIndex::sel_matches(idx.idents.items[i], idx.sels.items[s]) ? 1 : 0;
      if (hit[s]) isel[(size_t)i * SW + (s >> 6)] |= 1ull << (s & 63);
    }
    for (int32_t e = 0; e < E; ++e) {
      if (!hit[std::get<0>(idx.carry.items[e])]) continue;
      std::vector<uint64_t>& tgt = std::get<2>(idx.carry.items[e]) == KSIM_AFF_CARRY_ANTI ? ianti : iprio;
      tgt[(size_t)i * CW + (e >> 6)] |= 1ull << (e & 63);
    }
    for (int32_t w = 0; w < SW; ++w) live[i] |= isel[(size_t)i * SW + w] != 0;
    for (int32_t w = 0; w < CW; ++w) live[i] |= (ianti[(size_t)i * CW + w] | iprio[(size_t)i * CW + w]) != 0;
    if (keep_all) live[i] = 1;
  }
  t.remap.assign(I, 0);
  int32_t nl = 0;
  for (int32_t i = 0; i < I; ++i)
    if (live[i]) {
      t.remap[i] = ++nl;
      for (int32_t w = 0; w < SW; ++w) t.isel.push_back(isel[(size_t)i * SW + w]);
      for (int32_t w = 0; w < CW; ++w) { t.ianti.push_back(ianti[(size_t)i * CW + w]); t.iprio.push_back(iprio[(size_t)i * CW + w]); }
    }
  t.n_sel = NS; t.n_ident = nl; t.n_pair = P; t.n_carry = E; t.sw = SW; t.cw = CW;
  int64_t off = 0;
  for (const auto& pr : idx.pairs.items) {
    t.pair_sel.push_back(pr.first);
    t.pair_key.push_back(pr.second);
    t.pair_off.push_back(off);
    off += t.n_dom[pr.second];
  }
  t.cnt.assign(std::max<int64_t>(off, 1), 0);
  off = 0;
  for (const auto& e : idx.carry.items) {
    t.carry_key.push_back(std::get<1>(e));
    t.carry_kind.push_back(std::get<2>(e));
    t.carry_off.push_back(off);
    off += t.n_dom[std::get<1>(e)];
  }
  t.carried.assign(std::max<int64_t>(off, 1), 0);
  const int32_t A = (int32_t)idx.aclasses.items.size();
  t.n_aclass = A;
  t.ac.assign((size_t)A * 6, 0);
  for (int32_t a = 0; a < A; ++a) {
    const AClass& x = idx.aclasses.items[a];
    t.ac[a * 6 + 0] = (int32_t)t.terms.size(); t.ac[a * 6 + 1] = (int32_t)x.req.size();
    for (const Term& y : x.req) t.terms.push_back(ksim_aff_term{y.kind, y.pair, y.gate, y.exist, y.self_ok, 0, y.weight});
    t.ac[a * 6 + 2] = (int32_t)t.terms.size(); t.ac[a * 6 + 3] = (int32_t)x.pref.size();
    for (const Term& y : x.pref) t.terms.push_back(ksim_aff_term{y.kind, y.pair, y.gate, y.exist, y.self_ok, 0, y.weight});
    t.ac[a * 6 + 4] = (int32_t)t.carries.size(); t.ac[a * 6 + 5] = (int32_t)x.carries.size();
    for (const auto& y : x.carries) t.carries.push_back(ksim_aff_carry{y.first, 0, y.second});
    t.spread_pair.push_back(x.sp);
  }
  t.zone_key = idx.keys.find(ZONE_KEY);
  // the placed pods' contribution (NodeInfo.AddPod of every cached pod)
  for (const Placed& pl : placed) {
    const int64_t w = pl.node;
    for (int32_t cp = 0; cp < P; ++cp) {
      const int32_t s = t.pair_sel[cp];
      if (!((isel[(size_t)pl.ident * SW + (s >> 6)] >> (s & 63)) & 1ull)) continue;
      const int32_t d = t.dom[(size_t)t.pair_key[cp] * n + w];
      if (d >= 0) t.cnt[t.pair_off[cp] + d] += 1;
    }
    if (pl.aclass >= 0)
      for (int32_t j = t.ac[pl.aclass * 6 + 4]; j < t.ac[pl.aclass * 6 + 4] + t.ac[pl.aclass * 6 + 5]; ++j) {
        const int32_t e = t.carries[j].term;
        const int32_t d = t.dom[(size_t)t.carry_key[e] * n + w];
        if (d >= 0) t.carried[t.carry_off[e] + d] += t.carries[j].amount;
      }
  }
}

void aff_struct(const AffTables& a, int64_t n, int32_t hard_weight, ksim_affinity_tables* out) {
  ksim_affinity_tables& t = *out;
  t = ksim_affinity_tables{};
  t.n_keys = a.n_keys; t.n_sel = a.n_sel; t.n_ident = a.n_ident; t.n_pair = a.n_pair; t.n_carry = a.n_carry;
  t.n_aclass = a.n_aclass; t.n_terms = (int32_t)a.terms.size(); t.n_carries = (int32_t)a.carries.size();
  t.n_nodes = n;
  t.cnt_len = (int64_t)a.cnt.size(); t.carried_len = (int64_t)a.carried.size();
  t.hard_weight = hard_weight;
  t.sel_words = a.sw; t.carry_words = a.cw; t.zone_key = a.zone_key;
  t.dom = a.dom.data(); t.n_dom = a.n_dom.data();
  t.ident_sel = a.isel.data(); t.ident_anti = a.ianti.data(); t.ident_prio = a.iprio.data();
  t.pair_sel = a.pair_sel.data(); t.pair_key = a.pair_key.data(); t.pair_off = a.pair_off.data();
  t.carry_key = a.carry_key.data(); t.carry_kind = a.carry_kind.data(); t.carry_off = a.carry_off.data();
  t.ac = a.ac.data(); t.terms = a.terms.data(); t.carries = a.carries.data();
  t.cnt = a.cnt.data(); t.carried = a.carried.data();
  t.spread_pair = a.spread_pair.data();
}

int load_aff_tab(const AffTables& a, int64_t n, int32_t hard_weight, ksim_handle* h) {
  ksim_affinity_tables t;
  aff_struct(a, n, hard_weight, &t);
  return ksim_load_affinity(h, &t);
}

// ---------------------------------------------------------------- volume tables (volumes.py build_tables)
// NoVolumeZoneConflict per (volume class, label set) for the classes from `first` on, appended to
// ok[class][words] (words = ceil(L / 32)); *err: a class errs on some zone-labelled set
// (VolumeIndex.zone_verdicts).  Evaluated once per distinct (zone, region) constraint.
// Label sets grouped by their zone / region labels (the only labels NoVolumeZoneConflict reads),
// kept incrementally: label sets are only ever added, so a caller that keeps one ZoneGroups scans
// each label set once instead of once per volume class.
struct ZoneGroups {
  size_t upto = 0;
  std::map<std::vector<std::pair<Str, Str>>, int32_t> index;
  std::vector<std::vector<std::pair<Str, Str>>> cons;  // per group: its (key, value) constraints
  std::vector<std::vector<int32_t>> members;          // per group: its label sets
  void update(const Interner<LabelSetKey>& label_sets) {
    for (; upto < label_sets.items.size(); ++upto) {
      std::vector<std::pair<Str, Str>> c;
      for (const auto& l : label_sets.items[upto].labels)
        if (l.first == ZONE_LABEL || l.first == REGION_LABEL) c.push_back(l);
      auto it = index.find(c);
      if (it == index.end()) {
        it = index.emplace(c, (int32_t)cons.size()).first;
        cons.push_back(c);
        members.emplace_back();
      }
      members[it->second].push_back((int32_t)upto);
    }
  }
};

void vol_zone_verdicts(const VolumeIndex& vi, ZoneGroups& groups, const Interner<LabelSetKey>& label_sets, size_t first,
                       std::vector<uint32_t>* ok, bool* err) {
  groups.update(label_sets);
  const int32_t L = (int32_t)label_sets.items.size();
  const int32_t words = (L + 31) / 32;
  for (size_t k = first; k < vi.class_zone.size(); ++k) {
    const auto& zone = vi.class_zone[k];
    std::vector<uint32_t> row(words, 0);
    for (size_t g = 0; g < groups.cons.size(); ++g) {
      bool fits = true;
      if (!zone.empty() && !groups.cons[g].empty()) {
        std::map<Str, Str> cons(groups.cons[g].begin(), groups.cons[g].end());
        for (const ZoneEntry& z : zone) {
          if (z.kind == 2) continue;
          if (z.kind == 1) { *err = true; fits = false; break; }
          bool bad = false;
          for (const auto& kv : z.labels) {
            std::set<Str> zs;
            if (!zones_of(kv.second, &zs)) continue;
            auto it = cons.find(kv.first);
            if (!zs.count(it == cons.end() ? Str() : it->second)) { bad = true; break; }
          }
          if (bad) { fits = false; break; }
        }
      }
      if (fits)
        for (int32_t s : groups.members[g]) row[s >> 5] |= 1u << (s & 31);
    }
    ok->insert(ok->end(), row.begin(), row.end());
  }
}

void vol_zone_verdicts(const VolumeIndex& vi, const Interner<LabelSetKey>& label_sets, size_t first, std::vector<uint32_t>* ok,
                       bool* err) {
  ZoneGroups g;
  vol_zone_verdicts(vi, g, label_sets, first, ok, err);
}

// The small tables of ksim_volume_tables (keys, classes, refs) from an index.
struct VolSmall {
  std::vector<uint32_t> key_filter, vc_filter;
  std::vector<int32_t> vc;
  std::vector<ksim_vol_ref> refs;
};

void vol_small(const VolumeIndex& vi, VolSmall* t) {
  t->key_filter = vi.key_filter;
  t->vc.clear();
  t->refs.clear();
  for (const auto& cr : vi.class_refs) {
    t->vc.push_back((int32_t)t->refs.size());
    t->vc.push_back((int32_t)cr.size());
    for (const auto& e : cr) t->refs.push_back(ksim_vol_ref{e.first, e.second});
  }
  t->vc_filter = vi.class_filter;
}

// vol_small for a grow: only the keys / classes interned since `t` was built are appended (keys and
// classes keep their entries once interned), so the cost is the new entries, not every cached pod's.
void vol_small_append(const VolumeIndex& vi, VolSmall* t) {
  for (size_t k = t->key_filter.size(); k < vi.key_filter.size(); ++k) t->key_filter.push_back(vi.key_filter[k]);
  for (size_t c = t->vc_filter.size(); c < vi.class_refs.size(); ++c) {
    const auto& cr = vi.class_refs[c];
    t->vc.push_back((int32_t)t->refs.size());
    t->vc.push_back((int32_t)cr.size());
    for (const auto& e : cr) t->refs.push_back(ksim_vol_ref{e.first, e.second});
    t->vc_filter.push_back(vi.class_filter[c]);
  }
}

// ksim_load_volumes (full: with the slots) or ksim_grow_volumes (slots ignored) over the small tables.
int load_vol_tab(const VolSmall& v, int64_t n, int32_t S, const int32_t* max_vols, const std::vector<uint32_t>* zone_ok,
                 int32_t zone_words, bool full, const uint64_t* slots, const int32_t* slot_count, ksim_handle* h) {
  ksim_volume_tables t{};
  t.n_keys = (int32_t)v.key_filter.size();
  t.n_vclass = (int32_t)v.vc_filter.size();
  t.n_refs = (int32_t)v.refs.size();
  t.vol_slots = S;
  t.n_nodes = n;
  for (int k = 0; k < 3; ++k) t.max_vols[k] = max_vols[k];
  t.key_filter = v.key_filter.data();
  t.vc = v.vc.data();
  t.vc_filter = v.vc_filter.data();
  t.refs = v.refs.data();
  if (zone_ok && zone_words) {
    t.zone_words = zone_words;
    t.zone_ok = zone_ok->data();
  }
  t.slots = slots;
  t.slot_count = slot_count;
  return full ? ksim_load_volumes(h, &t) : ksim_grow_volumes(h, &t);
}

// The listers' objects (what the volume predicates resolve PVCs through).
void add_pv(VolumeIndex* vi, const ksim_k8s_pv& x) {
  PV pv;
  for (int32_t i = 0; i < x.n_labels; ++i) pv.labels[S(x.labels[i].key)] = S(x.labels[i].value);
  pv.kind = x.kind;
  pv.id = S(x.id);
  pv.node_affinity = x.has_node_affinity != 0;
  vi->pvs[S(x.name)] = pv;
}

void add_pvc(VolumeIndex* vi, const ksim_k8s_pvc& x) {
  PVC pvc;
  pvc.volume_name = S(x.volume_name);
  pvc.has_sc = x.storage_class != nullptr;
  pvc.sc = S(x.storage_class);
  vi->pvcs[{S(x.namespace_), S(x.name)}] = pvc;
}

void add_storage_class(VolumeIndex* vi, const ksim_k8s_storage_class& x) { vi->scs[S(x.name)] = {x.binding_mode != nullptr, S(x.binding_mode)}; }

// getMaxVols (predicates.go:347-359): KUBE_MAX_PD_VOLS when it parses to a positive int
void default_max_vols(int32_t* mv) {
  const int32_t def[3] = {39, 16, 16};
  const char* e = getenv("KUBE_MAX_PD_VOLS");
  int64_t v = 0;
  const bool ok = e && *e && parse_i64(e, &v) && v > 0 && v <= INT32_MAX;
  for (int k = 0; k < 3; ++k)
    if (mv[k] <= 0) mv[k] = ok ? (int32_t)v : def[k];
}

// ---------------------------------------------------------------- FitError text (generic_scheduler.go:72-90)
const char* reason_text(int r) {
  static const char* const T[KSIM_NREASONS] = {
      "node(s) were not ready", "node(s) were out of disk space", "node(s) had unavailable network",
      "node(s) were unschedulable", "Insufficient pods", "Insufficient cpu", "Insufficient memory",
      "Insufficient alpha.kubernetes.io/nvidia-gpu", "Insufficient ephemeral-storage",
      "node(s) didn't match the requested hostname", "node(s) didn't have free ports for the requested pod ports",
      "node(s) didn't match node selector", "node(s) had taints that the pod didn't tolerate",
      "node(s) had memory pressure", "node(s) had disk pressure", "node(s) didn't have the requested labels",
      nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr,
      "node(s) didn't match pod affinity/anti-affinity", "node(s) didn't satisfy existing pods anti-affinity rules",
      "node(s) didn't match pod affinity rules", "node(s) didn't match pod anti-affinity rules",
      "node(s) had no available disk", "node(s) exceed max volume count", "node(s) had no available volume zone",
      "node(s) didn't match service affinity"};
  return (r >= 0 && r < KSIM_NREASONS) ? T[r] : nullptr;
}

// FitError.Error: "0/N nodes are available: " + the sorted "count reason" parts joined by ", " + ".".
Str fit_error_text(int64_t num_nodes, const int32_t* hist, const std::vector<Str>& scalar_names) {
  std::vector<Str> parts;
  for (int r = 0; r < KSIM_NREASONS; ++r) {
    if (!hist[r]) continue;
    Str why;
    if (r >= KSIM_R_INSUFFICIENT_SCALAR0 && r < KSIM_R_INSUFFICIENT_SCALAR0 + KSIM_MAX_SCALAR) {
      const size_t col = (size_t)(r - KSIM_R_INSUFFICIENT_SCALAR0);
      why = "Insufficient " + (col < scalar_names.size() ? scalar_names[col] : Str("?"));
    } else {
      why = reason_text(r) ? reason_text(r) : "?";
    }
    parts.push_back(std::to_string(hist[r]) + " " + why);
  }
  std::sort(parts.begin(), parts.end());
  Str out = "0/" + std::to_string(num_nodes) + " nodes are available: ";
  for (size_t i = 0; i < parts.size(); ++i) out += (i ? ", " : "") + parts[i];
  return out + ".";
}

}  // namespace

#endif  // KSIM_K8S_SEM_H
