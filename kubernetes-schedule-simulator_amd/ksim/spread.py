"""SelectorSpreadPriority / ServiceSpreadingPriority inputs: the selectors of the services,
ReplicationControllers, ReplicaSets and StatefulSets that select a pod.

Reference: getSelectors (vendor/k8s.io/kubernetes/pkg/scheduler/algorithm/priorities/metadata.go:82-114)
over the scheduler's informer-backed listers, whose selection rules are client-go's
(vendor/k8s.io/client-go/listers/core/v1/service_expansion.go:36-56 — a nil selector selects nothing;
replicationcontroller_expansion.go:39-66, extensions/v1beta1/replicaset_expansion.go:41-73,
apps/v1beta1/statefulset_expansion.go:41-80 — a pod without labels has no controller, an empty
selector selects nothing, an invalid one fails the whole lookup).  The simulator's listers are empty
(no services in its store, fake controller informers: pkg/scheduler/simulator.go:352-367), so there
every pod has no selector and the priority is MaxPriority on every node; callers with services or
controllers pass them here.

The device never evaluates a selector: a pod's selector list becomes one interned "spread selector"
of the affinity tables (ksim/affinity.py), matched per identity on the host, with a per-node counted
pair that every commit maintains.
"""
from __future__ import annotations

from . import labels


class SpreadListers:
    def __init__(self, services=(), rcs=(), rss=(), sss=()):
        self.services, self.rcs, self.rss, self.sss = list(services), list(rcs), list(rss), list(sss)
        self._memo = {}   # (namespace, labels, services_only) -> selectors: pods share few label sets

    def __bool__(self):
        return bool(self.services or self.rcs or self.rss or self.sss)

    @staticmethod
    def _set_selects(sel: dict, lab: dict) -> bool:
        """labels.Set(sel).AsSelectorPreValidated().Matches(pod labels)."""
        return all(k in lab and lab[k] == v for k, v in sel.items())

    def selectors(self, pod, services_only=False):
        """getSelectors: a list of selectors (ksim.labels form), in lister order."""
        md = pod.get("metadata") or {}
        ns, lab = md.get("namespace", ""), md.get("labels") or {}
        key = (ns, tuple(sorted(lab.items())), services_only)
        hit = self._memo.get(key)
        if hit is None:
            hit = self._memo[key] = self._selectors(ns, lab, services_only)
        return hit

    def _selectors(self, ns, lab, services_only):
        out = []
        for svc in self.services:
            sel = (svc.get("spec") or {}).get("selector")
            if (svc.get("metadata") or {}).get("namespace", "") == ns and sel is not None and self._set_selects(sel, lab):
                out.append(labels.from_set(sel))
        if services_only or not lab:
            return out
        for rc in self.rcs:
            sel = (rc.get("spec") or {}).get("selector") or {}
            if (rc.get("metadata") or {}).get("namespace", "") == ns and sel and self._set_selects(sel, lab):
                out.append(labels.from_set(sel))
        for objs in (self.rss, self.sss):
            found = []
            try:
                for o in objs:
                    if (o.get("metadata") or {}).get("namespace", "") != ns:
                        continue
                    sel = labels.from_label_selector((o.get("spec") or {}).get("selector"))
                    if sel is labels.NOTHING or len(sel) == 0 or not labels.matches(sel, lab):
                        continue
                    found.append(sel)
            except labels.SelectorError:
                found = []
            out.extend(found)
        return out
