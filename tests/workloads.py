"""Seeded random Kubernetes-shaped workloads for parity tests (small enough for the
pure-Python oracle)."""
import random


def rnd_nodes(rng, n, features=True, name_fmt="node-{i}"):
    nodes = []
    for i in range(n):
        cpu = rng.choice([1000, 2000, 4000, 8000])
        mem = rng.choice([2, 4, 8, 16]) * 1024 ** 3
        node = {"metadata": {"name": name_fmt.format(i=i), "labels": {}}, "spec": {},
                "status": {"allocatable": {"cpu": "%dm" % cpu, "memory": str(mem), "pods": str(rng.choice([3, 5, 110]))},
                           "conditions": [{"type": "Ready", "status": "True"}]}}
        if features:
            node["metadata"]["labels"] = {"tier": rng.choice("abc"), "disk": rng.choice(["ssd", "hdd"])}
            if rng.random() < 0.3:
                node["metadata"]["labels"]["rank"] = str(rng.randint(0, 9))
            r = rng.random()
            if r < 0.15:
                node["spec"]["taints"] = [{"key": "dedicated", "value": "gpu", "effect": "NoSchedule"}]
            elif r < 0.3:
                node["spec"]["taints"] = [{"key": "spot", "value": "true", "effect": "PreferNoSchedule"}]
            elif r < 0.35:
                node["spec"]["taints"] = [{"key": "spot", "value": "true", "effect": "PreferNoSchedule"},
                                          {"key": "old", "value": "", "effect": "PreferNoSchedule"}]
            r = rng.random()
            if r < 0.04:
                node["status"]["conditions"][0]["status"] = "False"
            elif r < 0.06:
                node["spec"]["unschedulable"] = True
            elif r < 0.08:
                node["status"]["conditions"].append({"type": "MemoryPressure", "status": "True"})
            elif r < 0.09:
                node["status"]["conditions"].append({"type": "DiskPressure", "status": "True"})
            if rng.random() < 0.2:
                node["status"]["allocatable"]["example.com/fpga"] = str(rng.randint(0, 4))
            if rng.random() < 0.1:
                node["status"]["allocatable"]["alpha.kubernetes.io/nvidia-gpu"] = str(rng.randint(0, 2))
        nodes.append(node)
    rng.shuffle(nodes)
    return nodes


def rnd_pod(rng, name, features=True):
    cpu = rng.choice(["100m", "250m", "500m", "1", "2", None])
    mem = rng.choice(["128Mi", "256Mi", "1Gi", "2Gi", None])
    req = {}
    if cpu:
        req["cpu"] = cpu
    if mem:
        req["memory"] = mem
    ctr = {"resources": {"requests": req}} if req else {}
    spec = {"containers": [ctr]}
    if rng.random() < 0.2:
        spec["containers"].append({"resources": {"requests": {"cpu": "100m"}}})
    if features:
        if rng.random() < 0.1:
            spec["initContainers"] = [{"resources": {"requests": {"cpu": "1500m", "memory": "512Mi"}}}]
        if rng.random() < 0.3:
            spec["nodeSelector"] = {"tier": rng.choice("abc")}
        if rng.random() < 0.1:
            spec["affinity"] = {"nodeAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": {
                "nodeSelectorTerms": [{"matchExpressions": [{"key": "disk", "operator": "In", "values": ["ssd"]}]},
                                      {"matchExpressions": [{"key": "rank", "operator": "Gt", "values": ["4"]}]}]}}}
        if rng.random() < 0.15:
            spec.setdefault("affinity", {}).setdefault("nodeAffinity", {})[
                "preferredDuringSchedulingIgnoredDuringExecution"] = [
                {"weight": 3, "preference": {"matchExpressions": [{"key": "disk", "operator": "In", "values": ["ssd"]}]}},
                {"weight": 1, "preference": {"matchExpressions": [{"key": "tier", "operator": "NotIn", "values": ["a"]}]}}]
        if rng.random() < 0.2:
            spec["containers"][0]["ports"] = [{"hostPort": rng.choice([8080, 9090, 10250]),
                                               "protocol": rng.choice(["TCP", "UDP", ""]),
                                               "hostIP": rng.choice(["", "0.0.0.0", "10.0.0.1"])}]
        if rng.random() < 0.2:
            spec["tolerations"] = [{"key": "dedicated", "operator": "Equal", "value": "gpu", "effect": "NoSchedule"}]
        if rng.random() < 0.1:
            spec.setdefault("tolerations", []).append({"key": "spot", "operator": "Exists"})
        if rng.random() < 0.05:
            spec["containers"][0].setdefault("resources", {}).setdefault("requests", {})["example.com/fpga"] = "1"
        if rng.random() < 0.03:
            spec["containers"][0].setdefault("resources", {}).setdefault("requests", {})["alpha.kubernetes.io/nvidia-gpu"] = "1"
        if rng.random() < 0.02:
            spec["nodeName"] = "node-%d" % rng.randint(0, 5)
    return {"metadata": {"name": name, "namespace": ""}, "spec": spec}


def rnd_workload(seed, n_nodes=24, n_pods=120, n_running=10, features=True):
    rng = random.Random(seed)
    nodes = rnd_nodes(rng, n_nodes, features)
    running = []
    for k in range(n_running):
        p = rnd_pod(rng, "run-%d" % k, features)
        p["spec"]["nodeName"] = rng.choice(nodes)["metadata"]["name"]
        running.append(p)
    pods = [rnd_pod(rng, "sim-%d" % k, features) for k in range(n_pods)]
    return nodes, running, pods


PREFER_AVOID = "scheduler.alpha.kubernetes.io/preferAvoidPods"
CONTROLLERS = [("ReplicationController", "rc-uid-1"), ("ReplicationController", "rc-uid-2"),
               ("ReplicaSet", "rs-uid-1"), ("ReplicaSet", "rs-uid-2"), ("StatefulSet", "ss-uid-1")]


def add_prefer_avoid(seed, nodes, pods, keep_preferred=False):
    """NodePreferAvoidPods inputs on a workload (own stream, the base workload unchanged): ~35 %
    of nodes carry a preferAvoidPods annotation naming one or two controllers (some with a
    case-varied field name, a few malformed), ~50 % of pods an ownerReference (controller or not,
    RC / RS / other kinds) — those pods drop preferred node-affinity terms, so a pod class never
    needs more than the kernels' 16 reduce classes."""
    import json
    rng = random.Random(seed * 7919 + 13)
    for x in nodes:
        r = rng.random()
        if r < 0.35:
            ents = [{"podSignature": {"podController": {"apiVersion": "v1", "kind": k, "name": "c", "uid": u,
                                                        "controller": True}}, "reason": "r"}
                    for k, u in rng.sample(CONTROLLERS, rng.choice([1, 1, 2]))]
            doc = {"preferAvoidPods": ents} if rng.random() < 0.8 else {"PreferAvoidPods": ents}
            x["metadata"].setdefault("annotations", {})[PREFER_AVOID] = json.dumps(doc)
        elif r < 0.38:
            x["metadata"].setdefault("annotations", {})[PREFER_AVOID] = "{not json"
    for p in pods:
        if rng.random() < 0.5:
            k, u = rng.choice(CONTROLLERS)
            ref = {"kind": k, "name": "c", "uid": u}
            if rng.random() < 0.85:
                ref["controller"] = True
            p["metadata"]["ownerReferences"] = [ref]
            # (TaintToleration x NodeAffinity weight x avoid) classes must stay <= 16 per pod class:
            # an owned pod keeps its required node affinity, not its preferred terms
            if not keep_preferred:  # keep_preferred: pod classes beyond 16 reduce classes (the wide decision)
                na = ((p["spec"].get("affinity") or {}).get("nodeAffinity") or {})
                na.pop("preferredDuringSchedulingIgnoredDuringExecution", None)
    return nodes, pods


# ----------------------------------------------------------------------------- inter-pod affinity
AFF_KEYS = ["kubernetes.io/hostname", "zone", "region", "rack"]
APPS = ["web", "db", "cache", "batch"]


def rnd_affinity_nodes(rng, n, name_fmt="node-{i}"):
    """Nodes with topology labels: hostname (missing on a few), zone / region (missing on
    some), a sparse rack label, and two nodes sharing one hostname value."""
    nodes = rnd_nodes(rng, n, features=False, name_fmt=name_fmt)
    for k, x in enumerate(nodes):
        lab = x["metadata"].setdefault("labels", {})
        name = x["metadata"]["name"]
        if rng.random() < 0.9:
            lab["kubernetes.io/hostname"] = name if k != 1 else nodes[0]["metadata"]["name"]
        if rng.random() < 0.85:
            lab["zone"] = "z%d" % rng.randint(0, 3)
        if rng.random() < 0.8:
            lab["region"] = "r%d" % rng.randint(0, 1)
        if rng.random() < 0.25:
            lab["rack"] = "k%d" % rng.randint(0, 5)
        if rng.random() < 0.05:
            x["metadata"]["labels"] = None
        x["status"]["allocatable"]["pods"] = "110"
    return nodes


def _rnd_selector(rng):
    r = rng.random()
    if r < 0.45:
        return {"matchLabels": {"app": rng.choice(APPS)}}
    if r < 0.6:
        return {"matchExpressions": [{"key": "app", "operator": "In", "values": rng.sample(APPS, 2)}]}
    if r < 0.7:
        return {"matchExpressions": [{"key": "app", "operator": "NotIn", "values": [rng.choice(APPS)]}]}
    if r < 0.8:
        return {"matchExpressions": [{"key": "tier", "operator": "Exists"}]}
    if r < 0.85:
        return {"matchExpressions": [{"key": "tier", "operator": "DoesNotExist"}]}
    if r < 0.92:
        return {"matchLabels": {"app": rng.choice(APPS), "tier": rng.choice(["fe", "be"])}}
    return {}


def _rnd_term(rng, required):
    t = {"labelSelector": _rnd_selector(rng), "topologyKey": rng.choice(AFF_KEYS)}
    if rng.random() < 0.15:
        t["namespaces"] = rng.sample(["", "ns1", "ns2"], rng.randint(1, 2))
    if not required and rng.random() < 0.05:
        t["topologyKey"] = ""                       # allowed on preferred terms: contributes nothing
    return t


def rnd_affinity_pod(rng, name, p_aff=0.6, resources=True):
    """A pod with labels / namespace drawn from small sets and, with probability p_aff, pod
    (anti-)affinity terms of every kind."""
    pod = rnd_pod(rng, name, features=False) if resources else {"metadata": {"name": name}, "spec": {"containers": [{}]}}
    md = pod["metadata"]
    md["namespace"] = rng.choice(["", "", "ns1", "ns2"])
    md["labels"] = {"app": rng.choice(APPS)}
    if rng.random() < 0.5:
        md["labels"]["tier"] = rng.choice(["fe", "be"])
    if rng.random() < 0.1:
        md["labels"] = {}
    if rng.random() >= p_aff:
        return pod
    aff = {}
    for sec in ("podAffinity", "podAntiAffinity"):
        if rng.random() < 0.6:
            s = {}
            if rng.random() < 0.5:
                s["requiredDuringSchedulingIgnoredDuringExecution"] = [_rnd_term(rng, True)
                                                                        for _ in range(rng.randint(1, 2))]
            if rng.random() < 0.6:
                s["preferredDuringSchedulingIgnoredDuringExecution"] = [
                    {"weight": rng.randint(1, 100), "podAffinityTerm": _rnd_term(rng, False)}
                    for _ in range(rng.randint(1, 2))]
            aff[sec] = s
    if aff:
        pod["spec"]["affinity"] = aff
    return pod


def rnd_affinity_workload(seed, n_nodes=20, n_pods=80, n_running=12, p_aff=0.6, resources=True):
    rng = random.Random(seed)
    nodes = rnd_affinity_nodes(rng, n_nodes)
    running = []
    for k in range(n_running):
        p = rnd_affinity_pod(rng, "run-%d" % k, p_aff, resources)
        p["metadata"]["uid"] = "run-%d" % k
        p["spec"]["nodeName"] = rng.choice(nodes)["metadata"]["name"]
        running.append(p)
    pods = [rnd_affinity_pod(rng, "sim-%d" % k, p_aff, resources) for k in range(n_pods)]
    return nodes, running, pods


ZONE = "failure-domain.beta.kubernetes.io/zone"


def volume_listers(resolvable_only=False):
    """PVs / PVCs in namespace "ns": c1 → EBS PV, c2 → GCE PV (zones a, b), c6 → Azure PV,
    c7 → NFS-like PV (counted by no filter, zone c); unless resolvable_only: c3 unbound, c4 bound to
    a missing PV, c5 absent (MaxPD counts all three as their own ids)."""
    pvs = [{"metadata": {"name": "pv-ebs"}, "spec": {"awsElasticBlockStore": {"volumeID": "e1"}}},
           {"metadata": {"name": "pv-gce", "labels": {ZONE: "a__b"}}, "spec": {"gcePersistentDisk": {"pdName": "g1"}}},
           {"metadata": {"name": "pv-az"}, "spec": {"azureDisk": {"diskName": "a1"}}},
           {"metadata": {"name": "pv-nfs", "labels": {ZONE: "c"}}, "spec": {"nfs": {"server": "s"}}}]
    pvcs = [{"metadata": {"name": n, "namespace": "ns"}, "spec": {"volumeName": v}}
            for n, v in (("c1", "pv-ebs"), ("c2", "pv-gce"), ("c6", "pv-az"), ("c7", "pv-nfs"))]
    claims = ["c1", "c2", "c6", "c7"]
    if not resolvable_only:
        pvcs += [{"metadata": {"name": "c3", "namespace": "ns"}, "spec": {"volumeName": ""}},
                 {"metadata": {"name": "c4", "namespace": "ns"}, "spec": {"volumeName": "gone"}}]
        claims += ["c3", "c4", "c5"]
    return pvs, pvcs, claims


def rnd_volume(rng, claims, ids=("d1", "d2", "d3", "d4", "d5", "d6", "e1", "g1")):
    k = rng.random()
    ro = rng.random() < 0.4
    nm = rng.choice(ids)
    if k < 0.2:
        return {"gcePersistentDisk": {"pdName": nm, "readOnly": ro}}
    if k < 0.4:
        return {"awsElasticBlockStore": {"volumeID": nm, "readOnly": ro}}
    if k < 0.5:
        return {"iscsi": {"iqn": nm, "readOnly": ro, "targetPortal": "10.0.0.1:3260"}}
    if k < 0.6:
        return {"rbd": {"monitors": rng.sample(["m1", "m2", "m3"], rng.randint(1, 2)), "pool": "rbd", "image": nm,
                        "readOnly": ro}}
    if k < 0.7:
        return {"azureDisk": {"diskName": nm, "diskURI": "uri"}}
    if k < 0.9:
        return {"persistentVolumeClaim": {"claimName": rng.choice(claims)}}
    return {"emptyDir": {}}


def rnd_volume_workload(seed, n_nodes=16, n_pods=120, n_running=14, zones=False, resolvable_only=False, p_vol=0.7):
    """Nodes (optionally zone-labelled), running and queued pods in namespace "ns" mixing every
    volume kind the volume predicates read, with the listers they resolve through."""
    rng = random.Random(1000 + seed)
    nodes = rnd_nodes(rng, n_nodes, features=False)
    for x in nodes:
        x["status"]["allocatable"]["pods"] = "110"
        if zones and rng.random() < 0.7:
            x["metadata"]["labels"][ZONE] = rng.choice(["a", "b", "c"])
    pvs, pvcs, claims = volume_listers(resolvable_only)

    def pod(name, nn=None):
        p = rnd_pod(rng, name, features=False)
        p["metadata"]["namespace"] = "ns"
        if rng.random() < p_vol:
            p["spec"]["volumes"] = [rnd_volume(rng, claims) for _ in range(rng.randint(1, 3))]
        if nn:
            p["spec"]["nodeName"] = nn
        return p
    running = [pod("run-%d" % k, rng.choice(nodes)["metadata"]["name"]) for k in range(n_running)]
    pods = [pod("pod-%d" % k) for k in range(n_pods)]
    return nodes, running, pods, pvs, pvcs


def rnd_spread_workload(seed, n_nodes=18, n_pods=120, n_running=16, zones=True):
    """Pods labelled app=a|b|c, tier=x|y in namespaces ns1 / ns2 (a few being deleted among the
    running ones), services / RCs / RSs / StatefulSets selecting subsets, nodes in zones."""
    rng = random.Random(2000 + seed)
    nodes = rnd_nodes(rng, n_nodes, features=False)
    for x in nodes:
        x["status"]["allocatable"]["pods"] = "110"
        if zones and rng.random() < 0.8:
            x["metadata"]["labels"]["failure-domain.beta.kubernetes.io/zone"] = rng.choice(["z1", "z2", "z3"])
            if rng.random() < 0.3:
                x["metadata"]["labels"]["failure-domain.beta.kubernetes.io/region"] = "r1"

    def pod(name, nn=None):
        p = rnd_pod(rng, name, features=False)
        p["metadata"]["namespace"] = rng.choice(["ns1", "ns1", "ns2"])
        lab = {}
        if rng.random() < 0.9:
            lab["app"] = rng.choice("abc")
        if rng.random() < 0.5:
            lab["tier"] = rng.choice("xy")
        p["metadata"]["labels"] = lab
        if nn:
            p["spec"]["nodeName"] = nn
            if rng.random() < 0.1:
                p["metadata"]["deletionTimestamp"] = "2018-01-01T00:00:00Z"
        return p
    running = [pod("run-%d" % k, rng.choice(nodes)["metadata"]["name"]) for k in range(n_running)]
    pods = [pod("pod-%d" % k) for k in range(n_pods)]
    md = lambda ns: {"namespace": ns, "name": "o%d" % rng.randrange(1000)}
    services = [{"metadata": md("ns1"), "spec": {"selector": {"app": "a"}}},
                {"metadata": md("ns2"), "spec": {"selector": {"app": "b", "tier": "x"}}},
                {"metadata": md("ns1"), "spec": {}}]                                    # nil selector
    rcs = [{"metadata": md("ns1"), "spec": {"selector": {"tier": "y"}}}]
    rss = [{"metadata": md("ns2"), "spec": {"selector": {"matchExpressions": [
        {"key": "app", "operator": "In", "values": ["a", "c"]}]}}}]
    sss = [{"metadata": md("ns1"), "spec": {"selector": {"matchLabels": {"app": "c"}}}}]
    return nodes, running, pods, dict(services=services, rcs=rcs, rss=rss, sss=sss)


def rnd_mixed_workload(seed, n_nodes=120, n_pods=900):
    """Every feature at once: volumes (all kinds, PVCs through the listers), spread selectors,
    zones, labels, taints, selectors, host ports — the launch kernels' full predicate chain."""
    rng = random.Random(3000 + seed)
    nodes = rnd_nodes(rng, n_nodes, features=True)
    for x in nodes:
        x["status"]["allocatable"]["pods"] = "110"
        if rng.random() < 0.8:
            x["metadata"]["labels"]["failure-domain.beta.kubernetes.io/zone"] = rng.choice(["z1", "z2", "z3", "z4"])
    pvs, pvcs, claims = volume_listers(resolvable_only=True)
    _, _, _, objs = rnd_spread_workload(seed, n_nodes=1, n_pods=0, n_running=0)

    def pod(name, nn=None):
        p = rnd_pod(rng, name, features=True)
        p["metadata"]["namespace"] = rng.choice(["ns", "ns1", "ns2"])
        p["metadata"]["labels"] = {"app": rng.choice("abc"), "tier": rng.choice("xy")}
        if rng.random() < 0.5:
            p["spec"]["volumes"] = [rnd_volume(rng, claims) for _ in range(rng.randint(1, 2))]
            p["metadata"]["namespace"] = "ns"   # where the listers' PVCs live
        if nn:
            p["spec"]["nodeName"] = nn
        return p
    running = [pod("run-%d" % k, rng.choice(nodes)["metadata"]["name"]) for k in range(n_nodes // 3)]
    pods = [pod("pod-%d" % k) for k in range(n_pods)]
    return nodes, running, pods, pvs, pvcs, objs


def rnd_svc_affinity_workload(seed, n_nodes=24, n_pods=120, mixed_labels=False, conflicting_running=False,
                              full_labels=False):
    """CheckServiceAffinity with services (predicates.go:980-1011): nodes labelled region / rack
    (some without, unless full_labels), services selecting app=a / app=b in ns1 and app=a in ns2, pods with app=a|b|c
    (mixed_labels: sometimes tier=x too, so lender sets overlap and may disagree) and sometimes a
    nodeSelector for region shared by the pods of one (namespace, app); running pods of the services
    placed consistently on one region / rack each, or (conflicting_running) anywhere."""
    rng = random.Random(4000 + seed)
    nodes = rnd_nodes(rng, n_nodes, features=False)
    for x in nodes:
        x["status"]["allocatable"]["pods"] = "110"
        lab = x["metadata"]["labels"]
        if full_labels or rng.random() < 0.85:
            lab["region"] = rng.choice(["r1", "r2"])
        if full_labels or rng.random() < 0.7:
            lab["rack"] = rng.choice(["k1", "k2", "k3", "k4"])

    def pod(name, ns=None, app=None):
        p = rnd_pod(rng, name, features=False)
        p["metadata"]["namespace"] = ns or rng.choice(["ns1", "ns1", "ns2"])
        lab = {"app": app or rng.choice("abc")}
        if mixed_labels and rng.random() < 0.3:
            lab["tier"] = "x"
        p["metadata"]["labels"] = lab
        sel = group_sel.get((p["metadata"]["namespace"], lab["app"]))   # a deployment's pods share one
        if sel:
            p["spec"]["nodeSelector"] = dict(sel)
        return p
    group_sel = {(ns, app): ({"region": rng.choice(["r1", "r2"])} if rng.random() < 0.5 else None)
                 for ns in ("ns1", "ns2") for app in "abc"}
    running = []
    for k, (ns, app) in enumerate([("ns1", "a"), ("ns1", "b"), ("ns2", "a")]):
        home = rng.choice(nodes)["metadata"]["labels"]
        same = [x for x in nodes if all(x["metadata"]["labels"].get(l) == home.get(l) for l in ("region", "rack"))]
        for j in range(rng.randrange(0, 3)):
            q = pod("run-%d-%d" % (k, j), ns, app)
            q["spec"].pop("nodeSelector", None)
            q["spec"]["nodeName"] = rng.choice(nodes if conflicting_running else same)["metadata"]["name"]
            running.append(q)
    pods = [pod("pod-%d" % k) for k in range(n_pods)]
    md = lambda ns: {"namespace": ns, "name": "s%d" % rng.randrange(1000)}
    services = [{"metadata": md("ns1"), "spec": {"selector": {"app": "a"}}},
                {"metadata": md("ns1"), "spec": {"selector": {"app": "b"}}},
                {"metadata": md("ns2"), "spec": {"selector": {"app": "a"}}}]
    return nodes, running, pods, services
