"""Scheduler Policy files (the simulator's Policy path, pkg/scheduler/simulator.go:382-421) mapped
onto the supported key sets.

Reference semantics (paths under vendor/k8s.io/kubernetes/pkg/scheduler/):
- decoding: api/v1/types.go Policy {predicates: [{name, argument}], priorities: [{name, weight,
  argument}], extenders, hardPodAffinitySymmetricWeight, alwaysCheckAllPredicates}; the
  compatibility goldens are algorithmprovider/defaults/compatibility_test.go.
- validation: api/validation/validation.go:32-38 — every priority weight in (0, MaxWeight),
  MaxWeight = MaxInt / MaxPriority (api/types.go:31-38); errors aggregated (all reported).
- CreateFromConfig (factory/factory.go:932-1001): no "predicates" key → DefaultProvider's
  predicates, no "priorities" key → DefaultProvider's priorities; custom predicates / priorities
  with arguments are registered under their own names (factory/plugins.go:199-239, 303-343).
- getFitPredicateFunctions adds the mandatory predicates (plugins.go:401-406): CheckNodeCondition
  (defaults.go:165).
- podFitsOnNode runs only keys present in predicatesOrdering (algorithm/predicates/predicates.go:
  129-138, core/generic_scheduler.go:467): a predicate registered under any other name is never
  evaluated.

Unsupported pieces raise Unsupported (never a silently different result): HTTP extenders,
alwaysCheckAllPredicates, CheckServiceAffinity without a serviceAffinity argument, custom priorities with arguments other than
labelPreference / serviceAntiAffinity
(ServiceAntiAffinity / NodeLabelPriority) and priority keys outside the supported set.
"""
from __future__ import annotations

import json

from . import labels
from .ingest import Unsupported
from .scheduler import DEFAULT_PREDICATES, DEFAULT_PRIORITIES, PREDICATE_BITS, TRIVIAL_PREDICATES

MAX_INT = (1 << 63) - 1          # api/types.go:32 (64-bit Go int)
MAX_PRIORITY = 10                # api/types.go:36
MAX_WEIGHT = MAX_INT // MAX_PRIORITY

# predicates.go:129-138
PREDICATES_ORDERING = ("CheckNodeCondition", "CheckNodeUnschedulable", "GeneralPredicates", "HostName",
                       "PodFitsHostPorts", "MatchNodeSelector", "PodFitsResources", "NoDiskConflict",
                       "PodToleratesNodeTaints", "PodToleratesNodeNoExecuteTaints", "CheckNodeLabelPresence",
                       "CheckServiceAffinity", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount",
                       "CheckVolumeBinding", "NoVolumeZoneConflict", "CheckNodeMemoryPressure", "CheckNodeDiskPressure",
                       "MatchInterPodAffinity")
MANDATORY_PREDICATES = ("CheckNodeCondition",)


class PolicyError(ValueError):
    """validation.ValidatePolicy / decoding errors."""


class Policy:
    """A decoded Policy: the predicate and priority entries as written (names, weights,
    arguments), plus the options CreateFromConfig reads."""

    def __init__(self, predicates=None, priorities=None, extenders=(), hard_pod_affinity_symmetric_weight=0,
                 always_check_all_predicates=False):
        self.predicates = predicates      # None: not given; else [(name, argument or None)]
        self.priorities = priorities      # None: not given; else [(name, weight, argument or None)]
        self.extenders = list(extenders)
        self.hard_pod_affinity_symmetric_weight = hard_pod_affinity_symmetric_weight
        self.always_check_all_predicates = always_check_all_predicates

    def as_dict(self):
        return {"predicates": self.predicates, "priorities": self.priorities}


def decode(text_or_obj) -> Policy:
    """A Policy from JSON text (or YAML, or an already-parsed dict)."""
    if isinstance(text_or_obj, (str, bytes)):
        try:
            obj = json.loads(text_or_obj)
        except ValueError:
            import yaml
            obj = yaml.safe_load(text_or_obj)
    else:
        obj = text_or_obj
    if not isinstance(obj, dict):
        raise PolicyError("policy: not an object")
    kind = obj.get("kind", "Policy")
    if kind != "Policy":
        raise PolicyError("policy: kind %r is not Policy" % kind)
    preds = None
    if obj.get("predicates") is not None:
        preds = [(p["name"], p.get("argument")) for p in obj["predicates"]]
    prios = None
    if obj.get("priorities") is not None:
        prios = [(p["name"], int(p.get("weight", 0)), p.get("argument")) for p in obj["priorities"]]
    return Policy(preds, prios, obj.get("extenders") or obj.get("extenderConfigs") or (),
                  int(obj.get("hardPodAffinitySymmetricWeight", 0) or 0),
                  bool(obj.get("alwaysCheckAllPredicates", False)))


def validate(policy: Policy):
    """validation.ValidatePolicy (api/validation/validation.go:32-64): all errors, aggregated."""
    errs = []
    for name, weight, _ in policy.priorities or ():
        if weight <= 0 or weight >= MAX_WEIGHT:
            errs.append("Priority %s should have a positive weight applied to it or it has overflown" % name)
    binders = 0
    managed = set()
    for e in policy.extenders:
        if e.get("prioritizeVerb") and int(e.get("weight", 0)) <= 0:
            errs.append("Priority for extender %s should have a positive weight applied to it" % e.get("urlPrefix"))
        if e.get("bindVerb"):
            binders += 1
        for r in e.get("managedResources") or ():
            name = r.get("name", "")
            if not labels.qualified_name(name):   # validateExtendedResourceName (validation.go:66-80)
                errs.append("%s is not a qualified name" % name)
            elif not is_extended_resource_name(name):
                errs.append("%s is an invalid extended resource name" % name)
            if name in managed:
                errs.append("Duplicate extender managed resource name %s" % name)
            managed.add(name)
    if binders > 1:
        errs.append("Only one extender can implement bind, found %d" % binders)
    if errs:
        # utilerrors.NewAggregate: one error prints alone, several as "[a, b]"
        raise PolicyError(errs[0] if len(errs) == 1 else "[" + ", ".join(errs) + "]")


def is_extended_resource_name(name: str) -> bool:
    """IsExtendedResourceName (K/pkg/apis/core/v1/helper/helpers.go:38-57)."""
    if "/" not in name or "kubernetes.io/" in name or name.startswith("requests."):
        return False
    return labels.qualified_name("requests." + name)


def key_sets(policy: Policy):
    """CreateFromConfig (factory.go:932-1001) → (predicate keys, [(priority, weight)], label
    presence argument or None) as the GPU path runs them."""
    validate(policy)
    if policy.extenders:
        raise Unsupported("policy: HTTP extenders are outside the supported key set")
    if policy.always_check_all_predicates:
        raise Unsupported("policy: alwaysCheckAllPredicates is outside the supported key set")
    label_presence = None
    if policy.predicates is None:
        preds = list(DEFAULT_PREDICATES)
    else:
        preds = []
        for name, arg in policy.predicates:
            if name not in PREDICATES_ORDERING:
                continue  # registered, but podFitsOnNode never evaluates it
            if arg:
                if name == "CheckNodeLabelPresence" and arg.get("labelsPresence") is not None:
                    lp = arg["labelsPresence"]
                    label_presence = (list(lp.get("labels") or []), bool(lp.get("presence", False)))
                    preds.append(name)
                    continue
                if name == "CheckServiceAffinity" and arg.get("serviceAffinity") is not None:
                    preds.append(name)   # its labels: service_affinity_labels(policy)
                    continue
                raise Unsupported("policy: predicate %r with argument %r is outside the supported key set" % (name, arg))
            if name == "CheckNodeLabelPresence":
                raise Unsupported("policy: CheckNodeLabelPresence needs a labelsPresence argument")
            if name not in PREDICATE_BITS and name not in TRIVIAL_PREDICATES:
                raise Unsupported("policy: predicate %r is outside the supported key set" % name)
            preds.append(name)
    for m in MANDATORY_PREDICATES:
        if m not in preds:
            preds.append(m)
    if policy.priorities is None:
        prios = list(DEFAULT_PRIORITIES)
    else:
        prios = {}
        for name, weight, arg in policy.priorities:
            if arg and _priority_argument(name, arg) is None:
                raise Unsupported("policy: priority %r with argument %r is outside the supported key set" % (name, arg))
            prios[name] = weight  # a repeated name re-registers it: the last weight wins (plugins.go:343)
        prios = list(prios.items())
    return preds, prios, label_presence


def service_affinity_labels(policy: Policy):
    """The labels of a CheckServiceAffinity predicate registered with a serviceAffinity argument
    (factory/plugins.go:199-239), or None."""
    out = None
    for name, arg in policy.predicates or []:
        if name == "CheckServiceAffinity" and arg and arg.get("serviceAffinity") is not None:
            out = list(arg["serviceAffinity"].get("labels") or [])
    return out


def _priority_argument(name, arg):
    """RegisterCustomPriorityFunction (factory/plugins.go:271-323): a labelPreference argument
    registers NodeLabelPriority (priorities/node_label.go), a serviceAntiAffinity argument the
    ServiceAntiAffinity priority (selector_spreading.go:180-275) under the policy's name."""
    if arg.get("labelPreference") is not None:
        lp = arg["labelPreference"]
        return ("labelPreference", lp.get("label", ""), bool(lp.get("presence", False)))
    if arg.get("serviceAntiAffinity") is not None:
        return ("serviceAntiAffinity", arg["serviceAntiAffinity"].get("label", ""))
    return None


def priority_arguments(policy: Policy):
    """{priority name: ("labelPreference", label, presence) | ("serviceAntiAffinity", label)} of the
    policy's custom priorities (the last registration of a name wins)."""
    out = {}
    for name, _, arg in policy.priorities or []:
        spec = _priority_argument(name, arg) if arg else None
        if spec is not None:
            out[name] = spec
        else:
            out.pop(name, None)
    return out


def load(path):
    with open(path) as f:
        return decode(f.read())
