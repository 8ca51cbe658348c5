"""Volume tables for the device (ksim_volume_tables, include/ksim.h): NoDiskConflict, the MaxPD
volume counts and NoVolumeZoneConflict as the kernels evaluate them.

Reference semantics (file:line under vendor/k8s.io/kubernetes/pkg/scheduler/algorithm/predicates/):
- isVolumeConflict / NoDiskConflict (predicates.go:220-285): GCE PD by PDName (read-only mounts
  share), AWS EBS by VolumeID (never shared), ISCSI by IQN (read-only share), RBD when the Ceph
  monitor lists overlap and pool / image match (read-only share).  Only inline volumes of the
  incoming and the placed pods take part.
- MaxPDVolumeCountChecker (:287-507): per filter (EBS VolumeID, GCE PDName, Azure DiskName) the
  distinct ids of the placed pods plus the incoming pod's ids not already mounted, against the
  limit (getMaxVols :347-359, KUBE_MAX_PD_VOLS).  A PVC counts through its bound PV's id; a PVC
  the listers cannot resolve (missing, unbound, PV missing) counts as its own id in every filter.
- VolumeZoneChecker (:539-633): the zone / region labels of the PVs behind the pod's PVCs against
  the node's; a function of (pod volumes, node label set), precomputed per volume class.

The simulator's PV / PVC / StorageClass listers are empty (its store only holds nodes and pods),
so by default every PVC is unresolved; callers may pass the objects.  Cases where the reference
returns an error instead of a verdict (a PVC without a claim name, a PVC VolumeZone or
VolumeBinding cannot resolve) are reported in `errors` for the scheduler to refuse with
Unsupported when the predicate that errs is configured.
"""
from __future__ import annotations

import os

import numpy as np

from . import abi

ZONE_LABEL = "failure-domain.beta.kubernetes.io/zone"      # kubelet/apis/well_known_labels.go:21
REGION_LABEL = "failure-domain.beta.kubernetes.io/region"  # :23
DEFAULT_MAX_VOLS = (39, 16, 16)                            # EBS, GCE PD, Azure Disk (predicates.go:93-103)
_FILTERS = (("awsElasticBlockStore", "volumeID", abi.VOL_EBS, "EBS"),
            ("gcePersistentDisk", "pdName", abi.VOL_GCE_PD, "GCE"),
            ("azureDisk", "diskName", abi.VOL_AZURE_DISK, "AZ"))
_ALL_FILTERS = abi.VOL_EBS | abi.VOL_GCE_PD | abi.VOL_AZURE_DISK


def _go_atoi(s):
    import re
    if not re.fullmatch(r"[+-]?[0-9]+", s or ""):
        return None
    v = int(s)
    return v if -(1 << 63) <= v < (1 << 63) else None


def max_vols(raw=None):
    """getMaxVols (predicates.go:347-359) for the three filters: KUBE_MAX_PD_VOLS when it parses to
    a positive int (one value for all three), else each default."""
    raw = os.environ.get("KUBE_MAX_PD_VOLS", "") if raw is None else str(raw)
    v = _go_atoi(raw) if raw != "" else None
    return tuple(v if v is not None and v > 0 else d for d in DEFAULT_MAX_VOLS)


def _name(o):
    return (o.get("metadata") or {}).get("name", "")


def _ns(o):
    return (o.get("metadata") or {}).get("namespace", "")


def _zones(v):
    """volumeutil.LabelZonesToSet (pkg/volume/util/util.go:357-376); None on a parse error."""
    out = set()
    for z in v.split("__"):
        t = z.strip()
        if t == "":
            return None
        out.add(t)
    return out


class VolumeIndex:
    """Interns volume keys and volume classes over the pods of one cluster."""

    def __init__(self, pvs=(), pvcs=(), storage_classes=()):
        self.pvs = {_name(x): x for x in pvs}
        self.pvcs = {(_ns(x), _name(x)): x for x in pvcs}
        self.storage_classes = {_name(x): x for x in storage_classes}
        self.keys = {}
        self.key_filter = []
        self.classes = {}
        self.class_refs = []      # per class: [(key, flags)]
        self.class_filter = []
        self.class_zone = []      # per class: [(pvc name, pv labels or an error marker)]
        self.errors = set()       # "claim_name", "zone", "binding" (see module doc)

    def _key(self, ident, filt):
        k = self.keys.get(ident)
        if k is None:
            k = self.keys[ident] = len(self.key_filter)
            self.key_filter.append(filt)
        return k

    def _pvc_target(self, ns, claim):
        """The PV behind a PVC as MaxPD resolves it (predicates.go:367-408): (kind, id, filter), or
        None when the PV is not of a counted kind."""
        pvc = self.pvcs.get((ns, claim))
        pv_name = ((pvc or {}).get("spec") or {}).get("volumeName", "")
        pv = self.pvs.get(pv_name) if pvc is not None and pv_name else None
        if pv is None:
            return ("PVC", ns, claim), _ALL_FILTERS
        spec = pv.get("spec") or {}
        for kind, field, filt, tag in _FILTERS:
            src = spec.get(kind)
            if src is not None:
                return (tag, src.get(field, "")), filt
        return None

    def refs(self, pod, queued=True):
        """(refs [(key, flags)], zone list, has_pvc) of one pod's volumes; `queued`: the pod is
        scheduled (its PVCs meet VolumeZone / VolumeBinding), not already placed."""
        ns = _ns(pod)
        out, zone, has_pvc = [], [], False
        for vol in (pod.get("spec") or {}).get("volumes") or []:
            gce, ebs = vol.get("gcePersistentDisk"), vol.get("awsElasticBlockStore")
            iscsi, rbd, az = vol.get("iscsi"), vol.get("rbd"), vol.get("azureDisk")
            claim = vol.get("persistentVolumeClaim")
            if gce is not None:
                ro = bool(gce.get("readOnly"))
                out.append((self._key(("GCE", gce.get("pdName", "")), abi.VOL_GCE_PD),
                            (abi.VOL_CONFLICT_RW | abi.VOL_READ_ONLY) if ro else abi.VOL_CONFLICT_ANY))
            elif ebs is not None:
                ro = bool(ebs.get("readOnly"))
                out.append((self._key(("EBS", ebs.get("volumeID", "")), abi.VOL_EBS),
                            abi.VOL_CONFLICT_ANY | (abi.VOL_READ_ONLY if ro else 0)))
            elif iscsi is not None:
                ro = bool(iscsi.get("readOnly"))
                out.append((self._key(("ISCSI", iscsi.get("iqn", "")), 0),
                            (abi.VOL_CONFLICT_RW | abi.VOL_READ_ONLY) if ro else abi.VOL_CONFLICT_ANY))
            elif rbd is not None:
                ro = bool(rbd.get("readOnly"))
                for m in dict.fromkeys(rbd.get("monitors") or []):   # haveOverlap: some monitor shared
                    out.append((self._key(("RBD", m, rbd.get("pool", ""), rbd.get("image", "")), 0),
                                (abi.VOL_CONFLICT_RW | abi.VOL_READ_ONLY) if ro else abi.VOL_CONFLICT_ANY))
            elif az is not None:
                out.append((self._key(("AZ", az.get("diskName", "")), abi.VOL_AZURE_DISK), 0))
            elif claim is not None:
                has_pvc = True
                name = claim.get("claimName", "")
                if name == "":
                    self.errors.add("claim_name")   # filterVolumes (:369-371), VolumeZone (:572-574)
                    zone.append("error")
                    continue
                t = self._pvc_target(ns, name)
                if t is not None:
                    out.append((self._key(*t), abi.VOL_VIA_PVC))
                if queued:
                    zone.append(self._zone_entry(ns, name))
                    self._binding_check(ns, name)
        return out, zone, has_pvc

    def _zone_entry(self, ns, claim):
        """What VolumeZoneChecker reads for one PVC (predicates.go:570-628): the PV's zone / region
        labels, "skip" for a WaitForFirstConsumer claim, or "error"."""
        pvc = self.pvcs.get((ns, claim))
        if pvc is None:
            return "error"
        spec = pvc.get("spec") or {}
        pv_name = spec.get("volumeName", "")
        if pv_name == "":
            sc = spec.get("storageClassName")
            if sc:
                cls = self.storage_classes.get(sc)
                if cls is not None:
                    mode = cls.get("volumeBindingMode")
                    if mode is None:
                        return "error"
                    if mode == "WaitForFirstConsumer":
                        return "skip"
            return "error"
        pv = self.pvs.get(pv_name)
        if pv is None:
            return "error"
        return tuple(sorted((k, v) for k, v in ((pv.get("metadata") or {}).get("labels") or {}).items()
                            if k in (ZONE_LABEL, REGION_LABEL)))

    def _binding_check(self, ns, claim):
        """VolumeBinding's FindPodVolumes (scheduler_binder.go:127-167, :290-320) is restated only
        for PVCs bound to a PV without node affinity (always satisfied); anything else errs or is
        outside the restatement."""
        pvc = self.pvcs.get((ns, claim))
        pv = self.pvs.get(((pvc or {}).get("spec") or {}).get("volumeName", "")) if pvc is not None else None
        if pv is None or (pv.get("spec") or {}).get("nodeAffinity") is not None:
            self.errors.add("binding")

    def pod_errors(self, pod, label_sets):
        """The error paths one pod to be scheduled would take (module doc), without interning:
        "claim_name", "binding", "zone" (an unresolvable PVC while some label set is zoned)."""
        errs = set()
        ns = _ns(pod)
        zoned = any(k in dict(ls) for ls in label_sets for k in (ZONE_LABEL, REGION_LABEL))
        for vol in (pod.get("spec") or {}).get("volumes") or []:
            claim = vol.get("persistentVolumeClaim")
            if claim is None:
                continue
            name = claim.get("claimName", "")
            if name == "":
                errs.add("claim_name")
                continue
            if zoned and self._zone_entry(ns, name) == "error":
                errs.add("zone")
            pvc = self.pvcs.get((ns, name))
            pv = self.pvs.get(((pvc or {}).get("spec") or {}).get("volumeName", "")) if pvc is not None else None
            if pv is None or (pv.get("spec") or {}).get("nodeAffinity") is not None:
                errs.add("binding")
        return errs

    def mounts_of(self, vclass):
        """(key, slot field) of every ref of a volume class: 0 read-write, 1 read-only, 2 via PVC."""
        return [(k, 2 if f & abi.VOL_VIA_PVC else 1 if f & abi.VOL_READ_ONLY else 0)
                for k, f in self.class_refs[vclass - 1]]

    def vclass(self, pod):
        """1 + the pod's volume class, 0 when no volume matters to the predicates."""
        refs, zone, has_pvc = self.refs(pod)
        if not refs and not has_pvc:
            return 0
        seen, flagged, filt = set(), [], 0
        for k, f in refs:
            kf = self.key_filter[k]
            if kf and k not in seen:
                f |= abi.VOL_NEW
            seen.add(k)
            filt |= kf
            flagged.append((k, f))
        key = (tuple(flagged), tuple(zone))
        c = self.classes.get(key)
        if c is None:
            c = self.classes[key] = len(self.class_refs)
            self.class_refs.append(flagged)
            self.class_filter.append(filt)
            self.class_zone.append(zone)
        return c + 1

    def zone_verdicts(self, label_sets, first=0):
        """NoVolumeZoneConflict per (class, label set): bit table [n_class - first][words] for the
        classes from `first` on, and whether one of them errs somewhere (predicates.go:559-628).
        Evaluated once per distinct (zone, region) constraint of the label sets; classes without
        PVCs pass everywhere."""
        L = len(label_sets)
        words = (L + 31) // 32
        ok = np.zeros((len(self.class_zone) - first, max(words, 1)), np.uint32)
        cons_of = [tuple(sorted((k, v) for k, v in dict(ls).items() if k in (ZONE_LABEL, REGION_LABEL)))
                   for ls in label_sets]
        groups = {}
        for s, c in enumerate(cons_of):
            groups.setdefault(c, []).append(s)
        full = np.zeros(max(words, 1), np.uint32)
        for s in range(L):
            full[s >> 5] |= np.uint32(1 << (s & 31))
        err = False
        for c, zone in enumerate(self.class_zone[first:]):
            if not zone:
                ok[c] = full
                continue
            for cons_t, members in groups.items():
                cons = dict(cons_t)
                fits = True
                if cons:
                    for z in zone:
                        if z == "skip":
                            continue
                        if z == "error":
                            err = True
                            fits = False
                            break
                        bad = False
                        for k, v in z:
                            zs = _zones(v)
                            if zs is not None and cons.get(k, "") not in zs:
                                bad = True
                                break
                        if bad:
                            fits = False
                            break
                if fits:
                    for s in members:
                        ok[c, s >> 5] |= np.uint32(1 << (s & 31))
        return ok[:, :words] if words else ok[:, :0], err

    def node_slots(self, n, running):
        """Initial per-node mounts of the running pods: {node: {key: [rw, ro, pvc]}}."""
        mounts = [dict() for _ in range(n)]
        for node, pod in running:
            refs, _, _ = self.refs(pod, queued=False)
            for k, f in refs:
                m = mounts[node].setdefault(k, [0, 0, 0])
                m[2 if f & abi.VOL_VIA_PVC else 1 if f & abi.VOL_READ_ONLY else 0] += 1
        return mounts


def build_tables(index: VolumeIndex, n, mounts, queued_classes, label_sets, max_limits=None, vol_slots=None,
                 zone=None):
    """The ksim_volume_tables arrays (a dict of numpy arrays and sizes).  mounts=None: no slot
    arrays (ksim_grow_volumes keeps the device's); zone: precomputed (zone_ok, zone_err)."""
    key_filter = np.asarray(index.key_filter, np.uint32)
    refs = [r for c in index.class_refs for r in c]
    vc = np.zeros((len(index.class_refs), 2), np.int32)
    off = 0
    for c, r in enumerate(index.class_refs):
        vc[c] = (off, len(r))
        off += len(r)
    ref_arr = np.zeros(len(refs), abi.VOL_REF_DTYPE)
    if refs:
        ref_arr["key"] = [k for k, _ in refs]
        ref_arr["flags"] = [f for _, f in refs]
    # slots: the largest initial node plus every distinct key the queue could bring to one node
    qkeys = set()
    for c in set(queued_classes):
        if c > 0:
            qkeys.update(k for k, _ in index.class_refs[c - 1])
    need = max([len(m) for m in (mounts or ())] + [0]) + len(qkeys)
    S = int(need if vol_slots is None else vol_slots)
    slots = np.zeros((S, n) if mounts is not None else (0, 0), np.uint64)
    count = np.zeros(n if mounts is not None else 0, np.int32)
    for i, m in enumerate(mounts or ()):
        if len(m) > S:
            raise abi.KsimError(abi.E_INVAL, "vol_slots too small for running pods")
        for s, (k, (rw, ro, pv)) in enumerate(m.items()):
            if rw > 0x7FF or ro > 0x7FF or pv > 0x3FF:
                raise abi.KsimUnsupported(abi.E_UNSUPPORTED, "more mounts of one volume on a node than a slot counts")
            slots[s, i] = (k << 32) | (pv << 22) | (ro << 11) | rw
        count[i] = len(m)
    zone_ok, zone_err = index.zone_verdicts(label_sets) if zone is None else zone
    return dict(key_filter=key_filter, vc=vc, vc_filter=np.asarray(index.class_filter, np.uint32), refs=ref_arr,
                zone_ok=np.ascontiguousarray(zone_ok), zone_words=int(zone_ok.shape[1]), zone_err=zone_err,
                slots=slots, slot_count=count, vol_slots=S, n_nodes=n, grow_only=mounts is None,
                max_vols=tuple(max_vols() if max_limits is None else max_limits))


def tables_struct(d, use_zone=True):
    """ksim_volume_tables over the arrays of build_tables (they must outlive the call)."""
    t = abi.VolumeTables()
    t.n_keys = len(d["key_filter"])
    t.n_vclass = len(d["vc"])
    t.n_refs = len(d["refs"])
    t.vol_slots = d["vol_slots"]
    t.n_nodes = d["n_nodes"]
    for k in range(3):
        t.max_vols[k] = int(d["max_vols"][k])
    t.key_filter = abi.ptr(d["key_filter"], abi.C.c_uint32)
    t.vc = abi.ptr(d["vc"], abi.C.c_int32)
    t.vc_filter = abi.ptr(d["vc_filter"], abi.C.c_uint32)
    t.refs = abi.vptr(d["refs"])
    if use_zone and d["zone_words"]:
        t.zone_words = d["zone_words"]
        t.zone_ok = abi.ptr(d["zone_ok"], abi.C.c_uint32)
    if not d.get("grow_only"):
        t.slots = abi.ptr(d["slots"], abi.C.c_uint64)
        t.slot_count = abi.ptr(d["slot_count"], abi.C.c_int32)
    return t
