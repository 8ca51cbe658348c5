"""Deterministic synthetic workloads of SURVEY.md §8(d) / BASELINE.md, generated straight
into the device layout (splitmix64, seed = config index) so million-pod queues need no
per-object Python work.  C2 (labels, taints, host ports, selectors) goes through the
object path (ingest.Cluster.from_objects) because its string semantics are the point.

C1: 1,500 nodes test-{i}.test.com (lexical != numeric order), 32 cpu / 128Gi / 110 pods,
    etc/pod.yaml pods (A: cpu 1, memory 1 byte; B: cpu 100, memory 1000) expanded
    A x 48,010 then B x 10 and popped LIFO, DefaultProvider.
C3: 100,000 nodes node-{i:07d}, cpu {16,32,64}, mem {64,128,256}Gi, 110 pods;
    1,000,000 pods cpu {100m,250m,500m,1,2,4} x mem {256Mi,...,8Gi};
    default predicates + LeastRequested(1) + BalancedResourceAllocation(1).
C4: C3 distributions at 1,000,000 nodes / 10,000,000 pods.
C5: C3 distributions at 20,000 nodes, policy sweep scenarios (wLR, wBRA, wMR).
"""
from __future__ import annotations

import numpy as np

from . import abi, scheduler
from .ingest import Cluster, Interner

GI = 1 << 30
MI = 1 << 20


def splitmix64(seed: int, n: int) -> np.ndarray:
    """n outputs of splitmix64 seeded with `seed` (vectorised, wrapping uint64)."""
    with np.errstate(over="ignore"):
        z = (np.uint64(seed) + np.uint64(0x9E3779B97F4A7C15) * np.arange(1, n + 1, dtype=np.uint64))
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def _pick(r: np.ndarray, choices) -> np.ndarray:
    c = np.asarray(choices)
    return c[(r % np.uint64(len(c))).astype(np.int64)]


def _single_class_tables(cl: Cluster):
    cl.label_sets.get("{}", {})
    cl.taint_sets.get("[]", [])
    cl.classes.get("{}", {})
    cl._build_tables()


def resource_cluster(names, alloc_cpu, alloc_mem, allowed_pods, pod_cpu, pod_mem) -> Cluster:
    """Cluster of Ready, untainted, unlabelled nodes and resource-only pods (one pod class).
    `names` must already be in bytewise order (checked)."""
    n = len(alloc_cpu)
    cl = Cluster()
    cl.ips.get("0.0.0.0")
    cl.protos.get("TCP")
    cl.names = names
    if names is not None:
        enc = [s.encode() for s in names[: min(n, 4096)]]
        assert enc == sorted(enc), "node names must be given in bytewise order"
    z = np.zeros(n, np.int64)
    cl.cols = dict(alloc_cpu=np.asarray(alloc_cpu, np.int64), alloc_mem=np.asarray(alloc_mem, np.int64),
                   alloc_gpu=z.copy(), alloc_eph=z.copy(), allowed_pods=np.asarray(allowed_pods, np.int32),
                   flags=np.zeros(n, np.uint32), label_set=np.zeros(n, np.int32), taint_set=np.zeros(n, np.int32),
                   alloc_scalar=np.zeros((0, n), np.int64), req_cpu=z.copy(), req_mem=z.copy(), req_gpu=z.copy(),
                   req_eph=z.copy(), nz_cpu=z.copy(), nz_mem=z.copy(), pod_count=np.zeros(n, np.int32),
                   req_scalar=np.zeros((0, n), np.int64), ports=np.zeros((0, n), np.uint64),
                   port_count=np.zeros(n, np.int32))
    m = len(pod_cpu)
    pods = np.zeros(m, abi.POD_DTYPE)
    pc, pm = np.asarray(pod_cpu, np.int64), np.asarray(pod_mem, np.int64)
    for f in ("req_cpu", "add_cpu", "nz_cpu"):
        pods[f] = pc
    for f in ("req_mem", "add_mem", "nz_mem"):
        pods[f] = pm
    pods["host"] = -1
    pods["flags"] = np.where((pc != 0) | (pm != 0), abi.POD_ANY_REQUEST, 0).astype(np.uint32)
    cl.pods = pods
    cl.pod_names = None
    _single_class_tables(cl)
    return cl


def c3_nodes(n_nodes=100_000, seed=3):
    r = splitmix64(seed, 2 * n_nodes)
    cpu = _pick(r[0::2], [16, 32, 64]) * 1000
    mem = _pick(r[1::2], [64, 128, 256]) * GI
    return cpu, mem


def c3_pods(n_pods=1_000_000, seed=3):
    r = splitmix64(seed + 1000, 2 * n_pods)
    cpu = _pick(r[0::2], [100, 250, 500, 1000, 2000, 4000])
    mem = _pick(r[1::2], [256 * MI, 512 * MI, 1 * GI, 2 * GI, 4 * GI, 8 * GI])
    return cpu, mem


def config_c3(n_nodes=100_000, n_pods=1_000_000, seed=3, names=True):
    """C3 (BASELINE.json configs[2]): returns (cluster, predicates, priorities)."""
    cpu, mem = c3_nodes(n_nodes, seed)
    pcpu, pmem = c3_pods(n_pods, seed)
    nm = ["node-%07d" % i for i in range(n_nodes)] if names else None
    cl = resource_cluster(nm, cpu, mem, np.full(n_nodes, 110, np.int32), pcpu, pmem)
    preds = list(scheduler.DEFAULT_PREDICATES)
    prios = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]
    return cl, preds, prios


def config_c4(n_nodes=1_000_000, n_pods=10_000_000, seed=4):
    return config_c3(n_nodes, n_pods, seed, names=False)


def config_c1(n_nodes=1500, n_a=48_010, n_b=10):
    """C1 (BASELINE.json configs[0]): README node naming, etc/pod.yaml pods, LIFO order."""
    names = sorted(("test-%d.test.com" % i for i in range(n_nodes)), key=lambda s: s.encode())
    cpu = np.full(n_nodes, 32_000, np.int64)
    mem = np.full(n_nodes, 128 * GI, np.int64)
    # expanded list = A x n_a then B x n_b; PodQueue pops from the end → B first
    pcpu = np.concatenate([np.full(n_b, 100_000), np.full(n_a, 1000)])
    pmem = np.concatenate([np.full(n_b, 1000), np.full(n_a, 1)])
    cl = resource_cluster(names, cpu, mem, np.full(n_nodes, 110, np.int32), pcpu, pmem)
    cl.pod_names = ["B-%d" % (n_b - 1 - i) for i in range(n_b)] + ["A-%d" % (n_a - 1 - i) for i in range(n_a)]
    p, q = scheduler.provider("DefaultProvider")
    return cl, p, q


def c1_objects(n_nodes=1500, n_a=48_010, n_b=10):
    """C1 as Kubernetes-shaped objects: the README's nodes test-{i}.test.com (32 cpu, 128Gi,
    110 pods, Ready) and etc/pod.yaml's SimulationPod list (A: cpu 1 / memory 1 x n_a, then
    B: cpu 100 / memory 1000 x n_b) expanded by ParseSimulationPod (cmd/app/options/options.go:73-99).
    Returns (nodes, expanded pod list); the simulator pops the list from the end (LIFO)."""
    from .scheduler import expand_simulation_pods
    nodes = [{"metadata": {"name": "test-%d.test.com" % i},
              "status": {"allocatable": {"cpu": "32", "memory": "128Gi", "pods": "110"},
                         "conditions": [{"type": "Ready", "status": "True"}]}} for i in range(n_nodes)]
    spec = [{"name": "A", "num": n_a, "pod": {"spec": {"containers": [
                {"name": "a", "resources": {"requests": {"cpu": "1", "memory": "1"}}}]}}},
            {"name": "B", "num": n_b, "pod": {"spec": {"containers": [
                {"name": "b", "resources": {"requests": {"cpu": "100", "memory": "1000"}}}]}}}]
    return nodes, expand_simulation_pods(spec)


def c2_objects(n_nodes=5000, n_pods=50_000, seed=2):
    """C2 (BASELINE.json configs[1]) as Kubernetes-shaped objects: heterogeneous
    nodes with labels, NoSchedule / PreferNoSchedule taints and a few NotReady / unschedulable
    ones; pods with nodeSelector, host ports, tolerations and some BestEffort.  Returns
    (nodes, pods) with pods in SCHEDULING order."""
    import random
    rng = random.Random(seed)
    nodes = []
    for i in range(n_nodes):
        node = {"metadata": {"name": "c2-node-%d" % i,  # lexical != numeric order
                             "labels": {"tier": rng.choice("abc"), "disk": rng.choice(["ssd", "hdd"])}},
                "spec": {},
                "status": {"allocatable": {"cpu": str(rng.choice([8, 16, 32, 64])),
                                           "memory": "%dGi" % rng.choice([32, 64, 128, 256]), "pods": "110"},
                           "conditions": [{"type": "Ready", "status": "True"}]}}
        r = rng.random()
        if r < 0.10:
            node["spec"]["taints"] = [{"key": "dedicated", "value": "gpu", "effect": "NoSchedule"}]
        elif r < 0.20:
            node["spec"]["taints"] = [{"key": "spot", "value": "true", "effect": "PreferNoSchedule"}]
        r = rng.random()
        if r < 0.01:
            node["status"]["conditions"][0]["status"] = "False"
        elif r < 0.02:
            node["spec"]["unschedulable"] = True
        nodes.append(node)
    ports = [8080, 9090] + list(range(10250, 10260))
    pods = []
    for k in range(n_pods):
        ctr = {}
        if rng.random() >= 0.05:  # 5% BestEffort: no requests at all
            ctr["resources"] = {"requests": {"cpu": rng.choice(["100m", "250m", "500m", "1", "2"]),
                                             "memory": rng.choice(["128Mi", "256Mi", "512Mi", "1Gi", "2Gi"])}}
        spec = {"containers": [ctr]}
        if rng.random() < 0.30:
            spec["nodeSelector"] = {"tier": rng.choice("abc")}
        if rng.random() < 0.20:
            ctr["ports"] = [{"containerPort": 80, "hostPort": rng.choice(ports), "protocol": "TCP"}]
        if rng.random() < 0.15:
            spec["tolerations"] = [{"key": "dedicated", "operator": "Equal", "value": "gpu", "effect": "NoSchedule"}]
        pods.append({"metadata": {"name": "c2-pod-%d" % k, "namespace": "default"}, "spec": spec})
    return nodes, pods


def config_c2(n_nodes=5000, n_pods=50_000, seed=2):
    """C2 through the object path (ingest.Cluster.from_objects): (cluster, predicates,
    priorities) of the DefaultProvider."""
    nodes, pods = c2_objects(n_nodes, n_pods, seed)
    cl = Cluster.from_objects(nodes, (), pods)
    p, q = scheduler.provider("DefaultProvider")
    return cl, p, q


ZONE = "failure-domain.beta.kubernetes.io/zone"


def c2x_objects(n_nodes=5000, n_pods=50_000, seed=6):
    """C2 extended with the launch-kernel features: the C2 nodes (70 % in one of four zones) and
    pods, of which 25 % mount volumes (inline GCE PD / EBS from a pool of 2,000 disks, read-only
    now and then, or a PVC bound to a zoned GCE PV), 10 % carry a required pod anti-affinity term on
    kubernetes.io/hostname, every pod labelled app=<one of 20> and selected by that app's service
    (SelectorSpread).  Returns (nodes, pods, pvs, pvcs, services), pods in SCHEDULING order."""
    import random
    rng = random.Random(seed)
    nodes, pods = c2_objects(n_nodes, n_pods, seed)
    for x in nodes:
        if rng.random() < 0.7:
            x["metadata"]["labels"][ZONE] = "z%d" % rng.randrange(4)
        x["metadata"]["labels"]["kubernetes.io/hostname"] = x["metadata"]["name"]
    pvs = [{"metadata": {"name": "pv-%d" % i, "labels": {ZONE: "z%d" % (i % 4)}},
            "spec": {"gcePersistentDisk": {"pdName": "pv-disk-%d" % i}}} for i in range(400)]
    pvcs = [{"metadata": {"name": "claim-%d" % i, "namespace": "default"}, "spec": {"volumeName": "pv-%d" % i}}
            for i in range(400)]
    services = [{"metadata": {"name": "svc-%d" % a, "namespace": "default"}, "spec": {"selector": {"app": "a%d" % a}}}
                for a in range(20)]
    for p in pods:
        app = "a%d" % rng.randrange(20)
        p["metadata"]["labels"] = {"app": app}
        r = rng.random()
        if r < 0.10:
            disk = "d%d" % rng.randrange(2000)
            p["spec"]["volumes"] = [{"name": "v", "gcePersistentDisk": {"pdName": disk, "readOnly": rng.random() < 0.3}}]
        elif r < 0.20:
            p["spec"]["volumes"] = [{"name": "v", "awsElasticBlockStore": {"volumeID": "e%d" % rng.randrange(2000)}}]
        elif r < 0.25:
            p["spec"]["volumes"] = [{"name": "v", "persistentVolumeClaim": {"claimName": "claim-%d" % rng.randrange(400)}}]
        if rng.random() < 0.10:
            p["spec"]["affinity"] = {"podAntiAffinity": {"requiredDuringSchedulingIgnoredDuringExecution": [
                {"labelSelector": {"matchLabels": {"app": app}}, "topologyKey": "kubernetes.io/hostname"}]}}
    return nodes, pods, pvs, pvcs, services


def config_c2x(n_nodes=5000, n_pods=50_000, seed=6):
    """C2x through the object path with its listers: (cluster, predicates, priorities, objects) of
    the DefaultProvider; objects = dict(nodes, pods, pvs, pvcs, services) for the oracle."""
    from .spread import SpreadListers
    nodes, pods, pvs, pvcs, services = c2x_objects(n_nodes, n_pods, seed)
    cl = Cluster.from_objects(nodes, (), pods, pvs=pvs, pvcs=pvcs, spread=SpreadListers(services=services))
    p, q = scheduler.provider("DefaultProvider")
    return cl, p, q, dict(nodes=nodes, pods=pods, pvs=pvs, pvcs=pvcs, services=services)


def c5_scenarios():
    """4,096 (wLR, wBRA, wMR) policy points; wMR = 0 means MostRequested absent."""
    out = []
    for a in range(1, 17):
        for b in range(1, 17):
            for c in range(0, 16):
                pri = [("LeastRequestedPriority", a), ("BalancedResourceAllocation", b)]
                if c:
                    pri.append(("MostRequestedPriority", c))
                out.append(pri)
    return out


def config_c5(n_nodes=20_000, n_pods=5_000, seed=5):
    cpu, mem = c3_nodes(n_nodes, seed)
    pcpu, pmem = c3_pods(n_pods, seed)
    names = ["node-%07d" % i for i in range(n_nodes)]
    cl = resource_cluster(names, cpu, mem, np.full(n_nodes, 110, np.int32), pcpu, pmem)
    return cl, list(scheduler.DEFAULT_PREDICATES), c5_scenarios()
