"""Label-selector semantics the scheduler uses on node labels, evaluated once per
(pod class, node label set) on the host; the device only reads the resulting bits.

- SelectorFromSet: AM/pkg/labels/selector.go:837-853 (an invalid key or value makes the
  whole selector Everything()).
- Requirement.Matches: selector.go:193-235 (In/NotIn/Exists/DoesNotExist/Gt/Lt).
- NodeSelectorRequirementsAsSelector: K/pkg/apis/core/v1/helper/helpers.go:215-245 (an
  empty requirement list is Nothing()).
- podMatchesNodeLabels / nodeMatchesNodeSelectorTerms: predicates.go:780-838.
"""
from __future__ import annotations

import re

_NAME = re.compile(r"(?:[A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9]")
_DNS_SUB = re.compile(r"[a-z0-9](?:[-a-z0-9]*[a-z0-9])?(?:\.[a-z0-9](?:[-a-z0-9]*[a-z0-9])?)*")
_VALUE = re.compile(r"(?:(?:[A-Za-z0-9][-A-Za-z0-9_.]*)?[A-Za-z0-9])?")
_INT = re.compile(r"[+-]?[0-9]+")
_I64 = (-(1 << 63), (1 << 63) - 1)

NOTHING = None  # sentinel selector that matches no label set


class SelectorError(ValueError):
    pass


def qualified_name(k: str) -> bool:
    """validation.IsQualifiedName."""
    if k.count("/") > 1:
        return False
    if "/" in k:
        prefix, name = k.split("/")
        if not prefix or len(prefix) > 253 or not _DNS_SUB.fullmatch(prefix):
            return False
    else:
        name = k
    return 0 < len(name) <= 63 and bool(_NAME.fullmatch(name))


def label_value_ok(v: str) -> bool:
    return len(v) <= 63 and bool(_VALUE.fullmatch(v))


def _int64(s: str) -> int:
    if not _INT.fullmatch(s):
        raise SelectorError("not an integer")
    v = int(s)
    if not _I64[0] <= v <= _I64[1]:
        raise SelectorError("out of int64 range")
    return v


def requirement(key: str, op: str, values) -> tuple:
    """labels.NewRequirement with its validation; returns (key, op, sorted values)."""
    values = list(values or [])
    if not qualified_name(key):
        raise SelectorError("invalid label key %r" % key)
    if op in ("In", "NotIn"):
        if not values:
            raise SelectorError("values set can't be empty")
    elif op in ("=", "==", "!="):
        if len(values) != 1:
            raise SelectorError("exact-match compatibility requires one single value")
    elif op in ("Exists", "DoesNotExist"):
        if values:
            raise SelectorError("values set must be empty for exists and does not exist")
    elif op in ("Gt", "Lt"):
        if len(values) != 1:
            raise SelectorError("exactly one value is required")
        _int64(values[0])
    else:
        raise SelectorError("operator %r is not recognized" % op)
    for v in values:
        if not label_value_ok(v):
            raise SelectorError("invalid label value %r" % v)
    return (key, op, tuple(sorted(values)))


def req_matches(req: tuple, labels: dict) -> bool:
    key, op, values = req
    has = key in labels
    if op in ("In", "=", "=="):
        return has and labels[key] in values
    if op in ("NotIn", "!="):
        return (not has) or labels[key] not in values
    if op == "Exists":
        return has
    if op == "DoesNotExist":
        return not has
    if op in ("Gt", "Lt"):
        if not has or len(values) != 1:
            return False
        try:
            lv = _int64(labels[key])
        except SelectorError:
            return False
        rv = _int64(values[0])
        return lv > rv if op == "Gt" else lv < rv
    return False


def from_set(sel: dict):
    """SelectorFromSet: list of requirements; [] = Everything()."""
    out = []
    for k, v in (sel or {}).items():
        try:
            out.append(requirement(k, "=", [v]))
        except SelectorError:
            return []
    return out


def from_node_selector_requirements(exprs):
    """NodeSelectorRequirementsAsSelector; NOTHING for an empty list; raises on error."""
    if not exprs:
        return NOTHING
    ops = {"In", "NotIn", "Exists", "DoesNotExist", "Gt", "Lt"}
    out = []
    for e in exprs:
        op = e.get("operator")
        if op not in ops:
            raise SelectorError("%r is not a valid node selector operator" % op)
        out.append(requirement(e.get("key", ""), op, e.get("values")))
    return out


def from_label_selector(ps):
    """metav1.LabelSelectorAsSelector (apimachinery/pkg/apis/meta/v1/helpers.go): nil → NOTHING,
    empty → Everything ([]), matchLabels as equality requirements, matchExpressions with the
    In / NotIn / Exists / DoesNotExist operators; raises SelectorError like the Go error path."""
    if ps is None:
        return NOTHING
    ml, me = ps.get("matchLabels") or {}, ps.get("matchExpressions") or []
    if not ml and not me:
        return []
    out = [requirement(k, "=", [ml[k]]) for k in sorted(ml)]
    for e in me:
        op = e.get("operator")
        if op not in ("In", "NotIn", "Exists", "DoesNotExist"):
            raise SelectorError("%r is not a valid pod selector operator" % op)
        out.append(requirement(e.get("key", ""), op, e.get("values")))
    return out


def matches(sel, labels: dict) -> bool:
    if sel is NOTHING:
        return False
    return all(req_matches(r, labels) for r in sel)


def node_selector_terms_match(terms, labels: dict) -> bool:
    for t in terms or []:
        try:
            sel = from_node_selector_requirements(t.get("matchExpressions"))
        except SelectorError:
            return False
        if matches(sel, labels):
            return True
    return False


def pod_matches_node_labels(spec: dict, labels: dict) -> bool:
    ns = spec.get("nodeSelector") or {}
    if ns and not matches(from_set(ns), labels):
        return False
    na = (spec.get("affinity") or {}).get("nodeAffinity")
    if na is not None:
        req = na.get("requiredDuringSchedulingIgnoredDuringExecution")
        if req is None:
            return True
        return node_selector_terms_match(req.get("nodeSelectorTerms"), labels)
    return True


def preferred_weight(spec: dict, labels: dict) -> int:
    """CalculateNodeAffinityPriorityMap count (node_affinity.go:34-75); raises on a bad term."""
    na = (spec.get("affinity") or {}).get("nodeAffinity") or {}
    count = 0
    for term in na.get("preferredDuringSchedulingIgnoredDuringExecution") or []:
        w = int(term.get("weight", 0))
        if w == 0:
            continue
        sel = from_node_selector_requirements((term.get("preference") or {}).get("matchExpressions"))
        if matches(sel, labels):
            count += w
    return count
