"""Per-pod drop-in: the scheduler cache + ScheduleAlgorithm surface over the device table.

The reference scheduler calls Schedule(pod, nodeLister) once per pod
(vendor/k8s.io/kubernetes/pkg/scheduler/algorithm/scheduler_interface.go:52-65, caller
scheduler.go:188-204) and then Scheduler.assume (scheduler.go:366-397) → cache.AssumePod
(schedulercache/cache.go:125).  Informer events keep the cache in sync
(factory/factory.go:596 addPodToCache, :613 updatePodInCache, :695 deletePodFromCache, :740
addNodeToCache, :755 updateNodeInCache, :841 deleteNodeFromCache → cache.go:230-393).

SchedulerCache mirrors that surface with the same method names, arguments and error behaviour
(cache.go's "already in added state", "not found in scheduler cache", ...), keeps what the
device cannot (pod identity, node names, interned strings, residual pods of removed nodes) and
drives libksim.so for everything on the hot path: one scan launch per Schedule
(ksim_schedule_one), one small kernel per pod / node event (ksim_pod_add / remove,
ksim_node_add / update / remove).  There is no CPU fallback: without the library or a device
every call raises.
"""
from __future__ import annotations

import bisect
import ctypes as C

import numpy as np

from . import abi, ingest, scheduler
from .ingest import Unsupported, _canon, _meta, _spec


class FitError(Exception):
    """core.FitError (generic_scheduler.go:51-90): NumAllNodes + the reason histogram."""

    def __init__(self, num_nodes, hist, scalar_names=()):
        self.num_nodes = num_nodes
        self.hist = np.asarray(hist, np.int32)
        super().__init__(scheduler.fit_error_message(num_nodes, self.hist, scalar_names))


def pod_key(pod):
    """getPodKey (node_info.go:497-503): the UID; pods without one are keyed by namespace/name."""
    md = _meta(pod)
    return md.get("uid") or "%s/%s" % (md.get("namespace", ""), md.get("name", ""))


class _Info:
    """What the host keeps per NodeInfo (cache.nodes entry): the node object (None after
    RemoveNode or before AddNode), the pods on it with their encodings, the pressure status
    SetNode carries over."""

    __slots__ = ("node", "pods", "mem", "disk")

    def __init__(self):
        self.node = None
        self.pods = {}
        self.mem = self.disk = None


class SchedulerCache:
    """schedulercache.Cache + genericScheduler of one device.  `predicates` / `priorities` are
    key sets and weights as a provider or Policy lists them (scheduler.provider / policy)."""

    def __init__(self, predicates, priorities, device=0, mode=abi.MODE_AUTO, last_node_index=0, port_slots=4,
                 pvs=(), pvcs=(), storage_classes=(), hard_weight=10, spread=None):
        """pvs / pvcs / storage_classes: what the PV / PVC / StorageClass listers hold (the volume
        predicates resolve PVCs through them); hard_weight: hardPodAffinitySymmetricWeight; spread:
        ksim.spread.SpreadListers for SelectorSpread (None: the simulator's empty listers)."""
        from .volumes import VolumeIndex
        self.predicates = list(predicates)
        self.prioritizers = list(priorities)
        self.spread = spread if spread else None
        self.cfg = scheduler.make_config(predicates, priorities, device, mode, True, last_node_index,
                                         spread=self.spread is not None)
        self.hard_weight = int(hard_weight)
        names = {n for n, _ in priorities}
        self._spread_services_only = "ServiceSpreadingPriority" in names and "SelectorSpreadPriority" not in names
        # inter-pod affinity / SelectorSpread tables are needed once any cached or scheduled pod has
        # terms or spread selectors; then every call reloads them over the cached pods
        self._aff_on = False
        self._aidx = None        # the persistent AffinityIndex (None: rebuild it; node events reset it)
        self._aff_sig = None     # its sizes at the last table load
        self._aff_remap = None
        self._aff_check = False  # an affinity pod was cached on an unlisted node: re-check on the next call
        self.aff_reloads = 0     # affinity table loads so far (the per-pod path's amortised cost)
        self._aff_tables = None  # the loaded affinity tables (host copy)
        self._aff_wanted = bool(self.cfg.predicates & abi.P_INTERPOD_AFFINITY or
                                ((self.cfg.weights[abi.W_INTERPOD] or self.cfg.weights[abi.W_SPREAD])
                                 and not self.cfg.no_priorities))
        self._need_na = any(n == "NodeAffinityPriority" for n, _ in self.prioritizers)
        self.h = abi.Handle(self.cfg)
        cl = self.cl = ingest.Cluster()
        # ImageLocalityPriority reads node / pod images: intern them into label sets / classes
        cl.image_locality = any(n == "ImageLocalityPriority" for n, _ in self.prioritizers)
        cl.ips.get("0.0.0.0")
        cl.protos.get("TCP")
        cl.label_sets.get(_canon({}), {})
        cl.taint_sets.get(_canon([]), [])
        cl.classes.get(ingest.pod_class_key({}), {})
        cl.volume_index = VolumeIndex(pvs, pvcs, storage_classes)
        cl._affinity_ok = True   # affinity pods: their tables are built here per call (_sync_affinity)
        self._vol_on = bool(self.cfg.predicates & scheduler.VOLUME_PREDICATE_BITS)
        self._vol_key = None     # what the loaded volume tables were built for (None: not loaded)
        self._vol_mounts = {}    # node name -> {key: [rw, ro, pvc]} of its cached pods (incremental)
        self._vol_max = 0        # an upper bound of the mounted keys on any node
        self._vol_S = 0          # vol_slots of the loaded tables
        self._vol_zone = None    # NoVolumeZoneConflict verdicts of the loaded classes
        self.vol_loads = self.vol_grows = 0
        self._vol_dirty = False  # a node event since: the library refuses calls until a reload
        self.names = []          # listed node names, ascending bytewise (= name rank)
        self._keys = []          # the same as bytes
        self._rank = None        # name -> rank (rebuilt lazily after node events)
        self.infos = {}          # name -> _Info
        self.pod_states = {}     # key -> (pod, node name)
        self.assumed = set()
        self._tables_for = None
        self._load_tables()
        S = abi.MAX_SCALAR       # scalar columns reserved up front (new names need no relayout)
        t = abi.NodeTable()
        t.n_nodes, t.n_scalar, t.port_slots = 0, S, port_slots
        self._empty = {k: np.zeros(1, np.int64) for k in ("i64",)}
        self.h.call("ksim_load_nodes", C.byref(t))

    # ------------------------------------------------------------------ interning / tables
    def _load_tables(self):
        cl = self.cl
        key = (len(cl.label_sets.items), len(cl.taint_sets.items), len(cl.classes.items))
        if key == self._tables_for:
            return
        self.tables, self.need, bad = ingest.build_class_tables(cl.label_sets.items, cl.taint_sets.items,
                                                                cl.classes.items)
        cl.bad_affinity_classes = set(bad)
        tables, na_add = scheduler.class_tables_for(self.tables, self.prioritizers)
        self.h.call("ksim_load_classes", C.byref(ingest.class_tables_struct(tables, na_add)))
        self._tables_for = key

    def _scalar_id(self, name):
        i = self.cl.scalar_names.get(name)
        if i >= abi.MAX_SCALAR:
            raise Unsupported("more than %d scalar resources" % abi.MAX_SCALAR)
        return i

    def _ranks(self):
        if self._rank is None:
            self._rank = {n: i for i, n in enumerate(self.names)}
        return self._rank

    def _encode(self, pod):
        """Pod → (ksim_pod record array of 1, ports, scalars); interns its class first."""
        compiled = ingest.container_requests(pod)
        pred, add = compiled[0], compiled[1]
        for name in list(pred.scalar) + list(add.scalar):
            self._scalar_id(name)
        row = np.zeros(1, abi.POD_DTYPE)
        ports, scalars = [], []
        self.cl.encode_pod(pod, compiled, row[0], ports, scalars, index=self._ranks())
        self._load_tables()
        cls = int(row[0]["cls"])
        if self._need_na and cls in self.cl.bad_affinity_classes:
            raise Unsupported("NodeAffinityPriority: a preferred node-affinity term does not parse")
        row[0]["flags"] |= self.need[cls]
        p = np.array(ports, np.uint64)
        s = np.array(scalars, abi.SCALAR_DTYPE) if scalars else np.zeros(0, abi.SCALAR_DTYPE)
        return row, p, s

    def _pod_args(self, enc):
        row, p, s = enc
        return (abi.vptr(row), abi.vptr(p) if len(p) else None, len(p), abi.vptr(s) if len(s) else None, len(s))

    # ------------------------------------------------------------------ volume tables
    def _mounts(self):
        """Per listed node (name-rank order) the mounts of its cached pods: {key: [rw, ro, pvc]}
        (kept incrementally by _mount)."""
        return [self._vol_mounts.get(name, {}) for name in self.names]

    def _mount(self, name, enc, sign):
        """NodeInfo.AddPod / RemovePod of a volume pod's mounts on node `name` (host view)."""
        vc = int(enc[0][0]["vol_class"])
        if not vc or not self._vol_on:
            return
        m = self._vol_mounts.setdefault(name, {})
        for k, j in self.cl.volume_index.mounts_of(vc):
            e = m.setdefault(k, [0, 0, 0])
            e[j] += sign
            if not any(e):
                del m[k]
        self._vol_max = max(self._vol_max, len(m))

    def _sync_volumes(self, need, enc=None):
        """Keep the device's volume tables current for a call.  First load (when a volume pod needs
        them) and after every node event (the library marks them stale): the full tables with the
        cached pods' mounts.  Otherwise, when a pod brings new volume keys / classes or needs more
        slots per node than loaded: ksim_grow_volumes with the small tables only — the device keeps
        every node's mounts (its commits and releases maintain them), so the call costs
        O(keys + classes), not O(cached pods) (schedulercache/cache.go:200-318)."""
        if not self._vol_on:
            return
        idx = self.cl.volume_index
        key = (len(idx.key_filter), len(idx.class_refs), len(self.cl.label_sets.items))
        vc = int(enc[0][0]["vol_class"]) if enc is not None else 0
        want = self._vol_max + (len(idx.class_refs[vc - 1]) if vc else 0)
        if not self._vol_dirty and self._vol_key is None and not need:
            return
        if not self._vol_dirty and self._vol_key is not None:
            if self._vol_key == key and want <= self._vol_S:
                return
            if self._vol_key[2] == key[2]:
                from .volumes import build_tables, tables_struct
                old_n = len(self._vol_zone[0])
                if key[1] > old_n:
                    ok, err = idx.zone_verdicts(self.cl.label_sets.items, first=old_n)
                    self._vol_zone = (np.concatenate([self._vol_zone[0], ok]), self._vol_zone[1] or err)
                S = max(self._vol_S, 2 * want)
                t = build_tables(idx, len(self.names), None, (), self.cl.label_sets.items, vol_slots=S, zone=self._vol_zone)
                self.vol_tables = t
                self.h.call("ksim_grow_volumes", C.byref(tables_struct(t, "NoVolumeZoneConflict" in self.predicates)))
                self._vol_key, self._vol_S = key, S
                self.vol_grows += 1
                return
        from .volumes import build_tables, tables_struct
        n = len(self.names)
        self._vol_zone = idx.zone_verdicts(self.cl.label_sets.items)
        S = max(2 * want, 8)
        self.vol_tables = build_tables(idx, n, self._mounts(), (), self.cl.label_sets.items, vol_slots=S,
                                       zone=self._vol_zone)
        self.h.call("ksim_load_volumes", C.byref(tables_struct(self.vol_tables, "NoVolumeZoneConflict" in self.predicates)))
        self._vol_key, self._vol_S = key, S
        self._vol_dirty = False
        self.vol_loads += 1

    def _spread_sels(self, pod):
        return self.spread.selectors(pod, self._spread_services_only) if self.spread is not None else []

    def _sync_affinity(self, enc, pod, extra):
        """Inter-pod affinity and SelectorSpread through the affinity tables (ksim/affinity.py),
        kept incrementally like predicateMetadata.AddPod / RemovePod (predicates/metadata.go:127-190)
        and the cache's NodeInfo updates (schedulercache/cache.go:200-318): the index of selectors,
        counted pairs, carried terms, identities and term classes persists across calls, the
        device keeps the counts (every ksim_pod_add / _remove / assume updates them), and the tables
        are rebuilt over the cached pods and reloaded only when the index grew by something the
        device tables must hold (a new selector, pair, carried term, term class, or an identity
        that some selector matches) or after a node event.  A call that interns nothing new costs
        O(the pod's terms), not O(cached pods).  The tables are needed once any pod has terms or
        spread selectors; before that identities change nothing."""
        from .affinity import AffinityIndex, has_pod_affinity
        if not self._aff_wanted:
            return
        sels = self._spread_sels(pod)
        if not self._aff_on:
            if not has_pod_affinity(pod) and not sels:
                return
            self._aff_on = True
        for attempt in (0, 1):
            fresh = self._aidx is None
            if fresh:
                self._aidx = AffinityIndex([_meta(self.infos[n].node).get("labels") for n in self.names], self.hard_weight)
                self._aff_sig = None
            idx = self._aidx
            me_ident = idx.ident(pod)
            me_class = idx.aclass(pod, sels)
            if self._aff_sig is not None and not self._aff_check and self._aff_grew_only_dead(idx):
                grown = len(idx.idents.items) - len(self._aff_remap)
                self._aff_remap = np.concatenate([self._aff_remap, np.zeros(grown, np.int32)])
                self._aff_sig = self._aff_signature(idx)
                break
            try:
                self._aff_rebuild(idx)
                break
            except Unsupported:
                if fresh or attempt:
                    raise
                # a long-lived index keeps every selector / term it has seen: retry from the live pods
                self._aidx = None
        enc[0][0]["aff_ident"] = self._aff_remap[me_ident]
        enc[0][0]["aff_class"] = me_class + 1

    @staticmethod
    def _aff_signature(idx):
        return (len(idx.sels.items), len(idx.pairs.items), len(idx.carry.items), len(idx.keys.items),
                len(idx.aclasses.items), len(idx.idents.items))

    def _aff_grew_only_dead(self, idx):
        """Nothing the device tables hold changed since the last load, except new identities that
        no selector matches (their ksim_pod.aff_ident is 0: they count toward nothing)."""
        sig = self._aff_signature(idx)
        if sig[:5] != self._aff_sig[:5]:
            return False
        for it in idx.idents.items[self._aff_sig[5]:]:
            if any(idx._matches(it, si) for si in idx.sels.items):
                return False
        return True

    def _aff_rebuild(self, idx):
        """Rebuild the tables over the pods cached on listed nodes and load them (counts from the
        host's view of the cache)."""
        from .affinity import has_pod_affinity, tables_struct
        ranks = self._ranks()
        cached = []
        for name, info in self.infos.items():
            for p, _ in info.pods.values():
                if name in ranks:
                    cached.append((ranks[name], p))
                elif has_pod_affinity(p):
                    # the reference's metadata then errors on the node-less NodeInfo (metadata.go:106-109)
                    raise Unsupported("a pod with inter-pod affinity terms cached on a node that is not listed")
        idents = [idx.ident(p) for _, p in cached]
        aclasses = [idx.aclass(p) for _, p in cached]
        tables, remap = idx.build([w for w, _ in cached], idents, aclasses)
        self._aff_tables = tables
        self.h.call("ksim_load_affinity", C.byref(tables_struct(tables)))
        self._aff_remap = remap
        self._aff_sig = self._aff_signature(idx)
        self._aff_check = False
        self.aff_reloads += 1

    def _check_volume_errors(self, pod):
        """The scheduler refuses a pod on which a configured volume predicate errs (ksim/volumes.py)."""
        errs = self.cl.volume_index.pod_errors(pod, self.cl.label_sets.items)
        keys = set(self.predicates)
        maxpd = keys & {"MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount"}
        if "claim_name" in errs and (maxpd or "NoVolumeZoneConflict" in keys):
            raise Unsupported("a PersistentVolumeClaim volume without a claim name (the volume predicates err)")
        if "binding" in errs and "CheckVolumeBinding" in keys:
            raise Unsupported("CheckVolumeBinding with a PVC that is not bound to a PV without node affinity")
        if "zone" in errs and "NoVolumeZoneConflict" in keys:
            raise Unsupported("NoVolumeZoneConflict with a PVC the listers cannot resolve on a zone-labelled cluster")

    # ------------------------------------------------------------------ node rows
    def _node_row(self, name, info, ns):
        cl = self.cl
        imgs = ns.images if cl.image_locality else None
        lid = cl.label_sets.get(ingest.label_set_key(ns.labels, ns.prefer_avoid, imgs),
                                ingest.LabelSet(ns.labels, ns.prefer_avoid, imgs))
        tid = cl.taint_sets.get(_canon(ns.taints), ns.taints)
        cl.prefer_avoid_nodes |= bool(ns.prefer_avoid)
        alloc_s = np.zeros(abi.MAX_SCALAR, np.int64)
        for k, v in ns.scalar.items():
            alloc_s[self._scalar_id(k)] = v
        self._load_tables()
        r = abi.NodeRow()
        r.alloc_cpu, r.alloc_mem, r.alloc_gpu, r.alloc_eph = ns.alloc
        r.allowed_pods, r.flags, r.label_set, r.taint_set = ns.allowed, ns.flags, lid, tid
        # pods already on the node (NodeInfo kept across RemoveNode / pods seen before AddNode)
        req_s = np.zeros(abi.MAX_SCALAR, np.int64)
        keys = {}
        req = [0, 0, 0, 0]
        nzc = nzm = 0
        for pod, enc in info.pods.values():
            d = enc[0][0]
            req[0] += int(d["add_cpu"]); req[1] += int(d["add_mem"])
            req[2] += int(d["add_gpu"]); req[3] += int(d["add_eph"])
            nzc += int(d["nz_cpu"]); nzm += int(d["nz_mem"])
            for sc in enc[2]:
                req_s[int(sc["col"])] += int(sc["add"])
            for k in enc[1]:
                keys[int(k)] = True
        r.req_cpu, r.req_mem, r.req_gpu, r.req_eph = req
        r.nz_cpu, r.nz_mem = nzc, nzm
        r.pod_count = len(info.pods)
        ports = np.array(list(keys), np.uint64)
        r.port_count = len(ports)
        r.alloc_scalar = abi.ptr(alloc_s, C.c_int64)
        r.req_scalar = abi.ptr(req_s, C.c_int64)
        r.ports = abi.ptr(ports, C.c_uint64) if len(ports) else None
        return r, (alloc_s, req_s, ports)

    def _info(self, name):
        info = self.infos.get(name)
        if info is None:
            info = self.infos[name] = _Info()
        return info

    def add_node(self, node):
        """cache.AddNode (cache.go:354-363) → NodeInfo.SetNode."""
        name = _meta(node).get("name", "")
        info = self._info(name)
        ns = ingest.node_static(node, info.mem, info.disk)
        row, keep = self._node_row(name, info, ns)
        if name in self._ranks():
            self.h.call("ksim_node_update", self._ranks()[name], C.byref(row))
        else:
            k = name.encode()
            rank = bisect.bisect_left(self._keys, k)
            self.h.call("ksim_node_add", rank, C.byref(row))
            self._keys.insert(rank, k)
            self.names.insert(rank, name)
            self._rank = None
        info.node, info.mem, info.disk = node, ns.mem_pressure, ns.disk_pressure
        self._vol_dirty = self._vol_key is not None
        self._aidx = None

    def update_node(self, old, new):
        """cache.UpdateNode (cache.go:366-375) → SetNode on the (possibly new) NodeInfo."""
        self.add_node(new)

    def remove_node(self, node):
        """cache.RemoveNode (cache.go:378-393): the node leaves the listed set; its NodeInfo
        stays while pods remain on it (their events may arrive later)."""
        name = _meta(node).get("name", "")
        if name not in self._ranks():
            raise KeyError("node %s is not in the cache" % name)
        rank = self._ranks()[name]
        self.h.call("ksim_node_remove", rank)
        del self.names[rank]
        del self._keys[rank]
        self._rank = None
        info = self.infos[name]
        info.node, info.mem, info.disk = None, "Unknown", "Unknown"
        if not info.pods:
            del self.infos[name]
        self._vol_dirty = self._vol_key is not None
        self._aidx = None

    # ------------------------------------------------------------------ pods
    def _add(self, pod, enc=None):                          # cache.go:200-207
        name = _spec(pod).get("nodeName", "")
        enc = enc if enc is not None else self._encode(pod)
        if name in self._ranks():
            self._sync_volumes(bool(enc[0][0]["vol_class"]), enc)
            self._sync_affinity(enc, pod, True)
            self.h.call("ksim_pod_add", self._ranks()[name], *self._pod_args(enc))
        elif self._aff_on:
            self._aff_check = True
        self._info(name).pods[pod_key(pod)] = (pod, enc)
        self._mount(name, enc, 1)

    def _remove(self, pod):                                 # cache.go:219-228
        name = _spec(pod).get("nodeName", "")
        info = self.infos.get(name)
        key = pod_key(pod)
        if info is None or key not in info.pods:
            raise KeyError("no corresponding pod %s in pods of node %s" % (_meta(pod).get("name"), name))
        cur, enc = info.pods[key]
        if name in self._ranks():
            self._sync_volumes(bool(enc[0][0]["vol_class"]))
            self._sync_affinity(enc, cur, False)
            self.h.call("ksim_pod_remove", self._ranks()[name], *self._pod_args(enc))
        info.pods.pop(key)
        self._mount(name, enc, -1)
        if not info.pods and info.node is None:
            del self.infos[name]
        if self._aff_tables is not None and self._aff_tables.get("svc_on"):
            # the device only ever ORs service-affinity disagreements in (ksim_svc_commit): rebuild
            # the tables (their conflict words from the pods still cached) at the next call, so a
            # disagreement that left with this pod stops refusing its service identity
            self._aff_check = True

    def assume_pod(self, pod):
        """cache.AssumePod (cache.go:125-143); pod.spec.nodeName is the chosen host."""
        key = pod_key(pod)
        if key in self.pod_states:
            raise KeyError("pod %s is in the cache, so can't be assumed" % key)
        self._add(pod)
        self.pod_states[key] = pod
        self.assumed.add(key)

    def add_pod(self, pod):
        """cache.AddPod (cache.go:230-262): confirms an assumed pod (moving it if it landed
        elsewhere) or adds a pod bound by someone else."""
        key = pod_key(pod)
        cur = self.pod_states.get(key)
        if cur is not None and key in self.assumed:
            if _spec(cur).get("nodeName") != _spec(pod).get("nodeName"):
                self._remove(cur)
                self._add(pod)
            self.assumed.discard(key)
            self.pod_states[key] = pod
        elif cur is None:
            self._add(pod)
            self.pod_states[key] = pod
        else:
            raise KeyError("pod %s was already in added state" % key)

    def update_pod(self, old, new):
        """cache.UpdatePod (cache.go:265-289) = removePod(old) + addPod(new)."""
        key = pod_key(old)
        if key not in self.pod_states or key in self.assumed:
            raise KeyError("pod %s is not added to scheduler cache, so cannot be updated" % key)
        self._remove(old)
        self._add(new)
        self.pod_states[key] = new

    def remove_pod(self, pod):
        """cache.RemovePod (cache.go:292-318)."""
        key = pod_key(pod)
        cur = self.pod_states.get(key)
        if cur is None or key in self.assumed:
            raise KeyError("pod %s is not found in scheduler cache, so cannot be removed from it" % key)
        self._remove(cur)
        del self.pod_states[key]

    def forget_pod(self, pod):
        """cache.ForgetPod (cache.go:170-197): an assumed pod whose binding failed (scheduler.go:412)
        leaves the cache."""
        key = pod_key(pod)
        cur = self.pod_states.get(key)
        if cur is not None and _spec(cur).get("nodeName") != _spec(pod).get("nodeName"):
            raise KeyError("pod %s was assumed on %s but assigned to %s" % (key, _spec(pod).get("nodeName"),
                                                                          _spec(cur).get("nodeName")))
        if cur is None or key not in self.assumed:
            raise KeyError("pod %s wasn't assumed so cannot be forgotten" % key)
        self._remove(pod)
        self.assumed.discard(key)
        del self.pod_states[key]

    # ------------------------------------------------------------------ Schedule
    def schedule(self, pod, assume=False):
        """genericScheduler.Schedule (generic_scheduler.go:112-167): the host name, or raises
        FitError / abi.NoNodesAvailable.  assume=True also runs Scheduler.assume
        (scheduler.go:366): the pod enters the cache on that host, as an assumed pod."""
        enc = self._encode(pod)
        if enc[0][0]["vol_class"]:
            self._check_volume_errors(pod)
        self._sync_volumes(bool(enc[0][0]["vol_class"]), enc)
        self._sync_affinity(enc, pod, True)
        res = abi.Result()
        self.h.call("ksim_schedule_one", *self._pod_args(enc), abi.SCHEDULE_ASSUME if assume else abi.SCHEDULE_ONLY,
                    C.byref(res))
        self.last_fit_nodes = res.fit_nodes
        if res.node < 0:
            raise FitError(len(self.names), list(res.reasons), self.cl.scalar_names.items)
        host = self.names[res.node]
        if assume:
            assumed = dict(pod)
            assumed["spec"] = dict(_spec(pod), nodeName=host)
            key = pod_key(assumed)
            if key in self.pod_states:
                raise KeyError("pod %s is in the cache, so can't be assumed" % key)
            # the device already holds the commit: record it host-side with the assumed encoding
            enc2 = (enc[0].copy(), enc[1], enc[2])
            enc2[0][0]["host"] = res.node
            self._info(host).pods[key] = (assumed, enc2)
            self._mount(host, enc2, 1)
            self.pod_states[key] = assumed
            self.assumed.add(key)
        return host

    def schedule_one(self, pod):
        """scheduleOne's schedule + assume (scheduler.go:431-484) for one pod: (host, None) or
        (None, FitError message)."""
        try:
            return self.schedule(pod, assume=True), None
        except FitError as e:
            return None, str(e)

    @property
    def last_node_index(self):
        v = C.c_uint64()
        self.h.call("ksim_get_counter", C.byref(v))
        return v.value

    def node_count(self):
        v = C.c_int64()
        self.h.call("ksim_node_count", C.byref(v))
        return v.value

    def node_state(self):
        """Dynamic columns read back from the device, in name-rank order."""
        n = len(self.names)
        S = abi.MAX_SCALAR
        out = dict(req_cpu=np.zeros(n, np.int64), req_mem=np.zeros(n, np.int64), req_gpu=np.zeros(n, np.int64),
                   req_eph=np.zeros(n, np.int64), nz_cpu=np.zeros(n, np.int64), nz_mem=np.zeros(n, np.int64),
                   pod_count=np.zeros(n, np.int32), req_scalar=np.zeros((S, n), np.int64),
                   port_count=np.zeros(n, np.int32))
        st = abi.NodeState()
        for k, ct in (("req_cpu", C.c_int64), ("req_mem", C.c_int64), ("req_gpu", C.c_int64), ("req_eph", C.c_int64),
                      ("nz_cpu", C.c_int64), ("nz_mem", C.c_int64), ("pod_count", C.c_int32),
                      ("req_scalar", C.c_int64), ("port_count", C.c_int32)):
            setattr(st, k, abi.ptr(out[k], ct))
        self.h.call("ksim_read_nodes", C.byref(st))
        return out

    def close(self):
        self.h.close()
