"""The volume tables ksim/volumes.py builds, evaluated by the kernels' logic (tests/volume_model.py),
against the object oracle's NoDiskConflict / MaxPD / NoVolumeZoneConflict (oracle/ksim_ref.py,
pinned by the reference's tests in test_oracle_golden.py): the goldens, and random clusters whose
pods mix every volume kind, read-only mounts, PVCs resolved and unresolved."""
import random

import pytest

import ksim_ref as R
import volume_model as M
from golden_util import case_id, load
from ksim import abi, ingest

WHICH = {"MaxEBSVolumeCount": abi.VOL_EBS, "MaxGCEPDVolumeCount": abi.VOL_GCE_PD,
         "MaxAzureDiskVolumeCount": abi.VOL_AZURE_DISK}


def _model_fits(cl, pred, pod_index=0, node=0, mounts=None):
    d = cl.volumes
    vc = int(cl.pods["vol_class"][pod_index])
    if vc == 0:
        return True
    mounts = M.slots_of(d, node) if mounts is None else mounts
    if pred == "NoDiskConflict":
        return not M.disk_conflict(d, vc, mounts)
    if pred in WHICH:
        return not M.max_volume_fail(d, vc, mounts, WHICH[pred])
    assert pred == "NoVolumeZoneConflict"
    return M.zone_ok(d, vc, int(cl.cols["label_set"][node]))


@pytest.mark.parametrize("c", load("volumes"), ids=case_id)
def test_golden_through_tables(c):
    mv = c["max_vols"]
    cl = ingest.Cluster.from_objects([c["node"]], c["pods"], [c["pod"]], pvs=c["pvs"], pvcs=c["pvcs"],
                                     max_vols=None if mv is None else (mv, mv, mv))
    if cl.volumes is None:   # no predicate volumes anywhere: every volume predicate is true
        assert c["fits"]
        return
    assert _model_fits(cl, c["predicate"]) == c["fits"]


KINDS = ("gce", "ebs", "iscsi", "rbd", "az", "pvc", "host")


def _rand_volume(rng, names):
    k = rng.choice(KINDS)
    ro = rng.random() < 0.4
    nm = rng.choice(names)
    if k == "gce":
        return {"gcePersistentDisk": {"pdName": nm, "readOnly": ro}}
    if k == "ebs":
        return {"awsElasticBlockStore": {"volumeID": nm, "readOnly": ro}}
    if k == "iscsi":
        return {"iscsi": {"iqn": nm, "readOnly": ro, "targetPortal": "t"}}
    if k == "rbd":
        return {"rbd": {"monitors": rng.sample(["m1", "m2", "m3", "m4"], rng.randint(0, 2)), "pool": rng.choice(["p", "q"]),
                        "image": nm, "readOnly": ro}}
    if k == "az":
        return {"azureDisk": {"diskName": nm, "diskURI": "u"}}
    if k == "pvc":
        return {"persistentVolumeClaim": {"claimName": rng.choice(["c1", "c2", "c3", "c4", "c5"])}}
    return {"hostPath": {"path": "/x"}}


def _listers(rng):
    """PVs / PVCs: c1 → EBS pv, c2 → GCE pv (zone a), c3 → unbound, c4 → missing PV, c5 absent."""
    pvs = [{"metadata": {"name": "pv-ebs"}, "spec": {"awsElasticBlockStore": {"volumeID": "v1"}}},
           {"metadata": {"name": "pv-gce", "labels": {R.ZONE_LABEL: "a__b"}}, "spec": {"gcePersistentDisk": {"pdName": "v2"}}}]
    pvcs = [{"metadata": {"name": "c1", "namespace": "ns"}, "spec": {"volumeName": "pv-ebs"}},
            {"metadata": {"name": "c2", "namespace": "ns"}, "spec": {"volumeName": "pv-gce"}},
            {"metadata": {"name": "c3", "namespace": "ns"}, "spec": {"volumeName": ""}},
            {"metadata": {"name": "c4", "namespace": "ns"}, "spec": {"volumeName": "gone"}}]
    return pvs, pvcs


@pytest.mark.parametrize("seed", range(8))
def test_random_verdicts_and_commits(seed):
    """Per (pod, node): every volume predicate's verdict from the tables equals the oracle's, on
    nodes holding random running pods, then again after committing pods through the model."""
    rng = random.Random(seed)
    names = ["v1", "v2", "v3", "v4", "v5", "v6"]
    nodes = []
    for i in range(6):
        labels = {}
        if rng.random() < 0.5:
            labels[R.ZONE_LABEL] = rng.choice(["a", "b", "c"])
        nodes.append({"metadata": {"name": "n%d" % i, "labels": labels},
                      "status": {"allocatable": {"cpu": "64", "memory": "64Gi", "pods": "200"}}})
    def pod(name, nn=None):
        vols = [_rand_volume(rng, names) for _ in range(rng.randint(0, 4))]
        spec = {"volumes": vols, "containers": [{"name": "c"}]}
        if nn:
            spec["nodeName"] = nn
        return {"metadata": {"name": name, "namespace": "ns"}, "spec": spec}
    running = [pod("r%d" % k, "n%d" % rng.randrange(6)) for k in range(14)]
    queued = [pod("q%d" % k) for k in range(12)]
    pvs, pvcs = _listers(rng)
    mv = rng.choice([None, 2, 3])
    cl = ingest.Cluster.from_objects(nodes, running, queued, pvs=pvs, pvcs=pvcs,
                                     max_vols=None if mv is None else (mv, mv, mv))
    if cl.volumes is None:
        return
    listers = R.VolumeListers(pvs, pvcs)
    preds = R.volume_predicates(listers, mv)
    infos = [R.NodeInfo(x) for x in sorted(nodes, key=lambda x: x["metadata"]["name"].encode())]
    for r in running:
        infos[cl.index[r["spec"]["nodeName"]]].add_pod(r)
    mounts = [M.slots_of(cl.volumes, i) for i in range(len(infos))]
    checked = 0
    for q, p in enumerate(queued):
        for i, ni in enumerate(infos):
            for key in ("NoDiskConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount", "MaxAzureDiskVolumeCount",
                        "NoVolumeZoneConflict"):
                try:
                    ok, _ = preds[key](p, ni)
                except R.PredicateError:
                    # the product refuses these inputs (ksim.scheduler.check_volume_support)
                    assert key in ("NoVolumeZoneConflict", "MaxEBSVolumeCount", "MaxGCEPDVolumeCount",
                                   "MaxAzureDiskVolumeCount")
                    if key == "NoVolumeZoneConflict":
                        assert cl.volumes["zone_err"]
                    continue
                assert _model_fits(cl, key, q, i, mounts[i]) == ok, (seed, q, i, key)
                checked += 1
        # place the pod on a random node: NodeInfo.AddPod and the model's commit
        i = rng.randrange(len(infos))
        placed = dict(p, spec=dict(p["spec"], nodeName=infos[i].name))
        infos[i].add_pod(placed)
        vc = int(cl.pods["vol_class"][q])
        if vc:
            M.commit(mounts[i], cl.volumes, vc)
    assert checked > 100
    # and NodeInfo.RemovePod of running pods through the model's release
    for r in running:
        i = cl.index[r["spec"]["nodeName"]]
        refs, _, _ = cl.volume_index.refs(r, queued=False)
        for k, f in refs:
            j = 2 if f & abi.VOL_VIA_PVC else 1 if f & abi.VOL_READ_ONLY else 0
            mounts[i][k][j] -= 1
            if sum(mounts[i][k]) == 0:
                del mounts[i][k]
        infos[i].remove_pod(r)
    for q, p in enumerate(queued):
        for i, ni in enumerate(infos):
            ok, _ = preds["NoDiskConflict"](p, ni)
            assert _model_fits(cl, "NoDiskConflict", q, i, mounts[i]) == ok


@pytest.mark.parametrize("seed", range(4))
def test_grown_tables_match_full_build(seed):
    """What the per-pod path hands ksim_grow_volumes (build_tables without mounts, zone verdicts
    of the new classes appended to the old ones) equals the full build's class-side arrays, and
    carries no slot arrays."""
    import numpy as np
    from ksim.volumes import build_tables, tables_struct
    rng = random.Random(100 + seed)
    names = ["v1", "v2", "v3", "v4", "v5", "v6"]
    nodes = []
    for i in range(5):
        labels = {R.ZONE_LABEL: rng.choice(["a", "b", "c"])} if rng.random() < 0.6 else {}
        nodes.append({"metadata": {"name": "n%d" % i, "labels": labels},
                      "status": {"allocatable": {"cpu": "64", "memory": "64Gi", "pods": "200"}}})
    queued = [{"metadata": {"name": "q%d" % k, "namespace": "ns"},
               "spec": {"volumes": [_rand_volume(rng, names) for _ in range(rng.randint(1, 3))],
                        "containers": [{"name": "c"}]}} for k in range(16)]
    pvs, pvcs = _listers(rng)
    cl = ingest.Cluster.from_objects(nodes, (), queued, pvs=pvs, pvcs=pvcs)
    if cl.volumes is None:
        return
    idx, ls = cl.volume_index, cl.label_sets.items
    full_ok, full_err = idx.zone_verdicts(ls)
    k = len(idx.class_refs) // 2
    head_ok, head_err = idx.zone_verdicts(ls, first=0)
    tail_ok, tail_err = idx.zone_verdicts(ls, first=k)
    assert np.array_equal(np.concatenate([head_ok[:k], tail_ok]), full_ok)
    full = build_tables(idx, cl.n_nodes, [{} for _ in range(cl.n_nodes)], (), ls, vol_slots=8)
    grow = build_tables(idx, cl.n_nodes, None, (), ls, vol_slots=8, zone=(full_ok, full_err))
    for name in ("key_filter", "vc", "vc_filter", "zone_ok"):
        assert np.array_equal(full[name], grow[name]), name
    assert np.array_equal(full["refs"], grow["refs"])
    t = tables_struct(grow)
    assert not t.slots and not t.slot_count and t.vol_slots == 8
    t_full = tables_struct(full)
    assert t_full.slots and t_full.slot_count
