"""Benchmark of the MI355X per-pod scheduling cycle on BASELINE.json's headline workload.

Workload (BASELINE.json configs[2], SURVEY.md §8d "C3", the default; --workload c2 / c4 / c5
run the other configs the same way): 100,000 nodes, a 1,000,000-pod queue of mixed sizes,
default predicates + LeastRequested(1) + BalancedResourceAllocation(1).  A "step" is one
ksim_schedule() call over the next slice of the queue (each pod: predicates on every node,
priorities, selectHost, commit — strictly one after another), with the node table and pod
queue resident in HBM.  The K timed steps cover the WHOLE queue (slice = queue / K pods); the
W warmup steps run the head of the queue on a separate copy of the cluster first, so the
timed run starts from the empty cluster and ends at the queue's last pod.

N GPUs (torchrun, one process per GPU):
  * headline `value` (--shard nodes, the default): ONE 100k-node cluster split into N
    contiguous name-rank shards, one per GPU; each pod is decided jointly through the per-pod
    exchange over xGMI (ksim_shard_*), the owning rank commits.  pods/s of that one cluster
    (scaling "strong"); placements checked against a single-GPU run of the same queue.
  * `replicas`: every rank schedules its own cluster under its own LeastRequested weight (a
    what-if sweep, no data-path collective; scaling "weak").  --shard replicas makes it the
    headline instead.

The JSON line carries the roofline of the dominant kernel (algorithmic bytes per launch ÷ the
HIP-event launch duration measured on the library's stream, against the 8 TB/s HBM peak; null
for tree mode, whose kernel does not read the table per pod) and a cpu_baseline: the C port of
the Go path (oracle/cpu_ref.c) timed on the host on bounded prefixes of the same queue at 1, 16
and all threads, its placements equal to the GPU's for the same prefix ("parity").
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [os.path.join(ROOT, "kubernetes-schedule-simulator_amd")]

BYTES_PER_NODE_EVAL = 60   # 6 x i64 + 2 x i32 + u32 flags, resource-only pods
HBM_PEAK_GBS = 8000.0      # MI355X_MICROARCH.md: 8.0 TB/s spec


def pmc_traffic(workload, evals_per_launch):
    """HBM bytes per launch of the dominant kernel from the committed PMC profile
    (profiles/pmc_<workload>.json: FETCH_SIZE x2 + WRITE_SIZE per node-eval, collected with
    tools/gpu_pmc.sh / tools/gpu_c5.sh as MI355X_MICROARCH.md prescribes), or None."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "pmc_%s.json" % workload)))
        return round(d["hbm_bytes_per_node_eval"] * evals_per_launch / 1e9, 6)  # GB per launch
    except (OSError, KeyError, ValueError):
        return None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None, help="timed ksim_schedule calls (default: c3 20, c2 9, c4 10)")
    ap.add_argument("--warmup", type=int, default=None, help="untimed calls on a separate cluster copy (default 2)")
    ap.add_argument("--batch", type=int, default=None,
                    help="pods per step (default: c3 / c2 the whole queue over the timed steps, c4 512)")
    ap.add_argument("--nodes", type=int, default=None, help="default: c3 100,000, c2 5,000, c4 1,000,000")
    ap.add_argument("--pods", type=int, default=None, help="queue length (default: c3 1M, c2 50k, c4 as needed)")
    ap.add_argument("--mode", default="auto", choices=["auto", "launch", "persistent", "tree"])
    ap.add_argument("--no-tree", dest="tree", action="store_false",
                    help="skip the tree-mode line measured beside the scan (c3/c4)")
    ap.add_argument("--cpu-sample", type=int, default=30000,
                    help="most pods in a CPU-baseline prefix (0 = skip); each leg is sized to ~10 s of CPU work")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--workload", default="c3", choices=["c3", "c2", "c2x", "c4", "c5"],
                    help="c3: the headline metric (default); c2: 5k heterogeneous nodes with selectors, "
                         "ports and taints; c4: 1M nodes; c5: the 4,096-scenario policy sweep")
    ap.add_argument("--scenarios", type=int, default=4096, help="c5: total scenarios (split across ranks)")
    ap.add_argument("--sweep-nodes", type=int, default=20_000, help="c5: nodes per scenario")
    ap.add_argument("--sweep-form", default="auto", choices=["auto", "scan"],
                    help="c5: auto = tree form when eligible; scan = the per-scenario scan kernel")
    ap.add_argument("--sweep-pods", type=int, default=5000, help="c5: pods scheduled in every scenario")
    ap.add_argument("--shard", default="nodes", choices=["nodes", "replicas", "none"],
                    help="N>1 headline: one node-sharded cluster (strong, default) or per-rank replicas "
                         "(weak); the other one is measured beside it unless 'none'")
    ap.add_argument("--replica-pods", type=int, default=200_000, help="N>1: queue prefix of the replica side line")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on device 0 (gloo), grids split so the "
                         "ranks' persistent kernels are co-resident")
    a = ap.parse_args()
    d = WORKLOADS[a.workload]
    for k in ("steps", "warmup", "nodes", "pods"):
        if getattr(a, k) is None:
            setattr(a, k, d.get(k))
    if a.batch is None:
        a.batch = d.get("batch") or -(-a.pods // a.steps)
    if a.pods is None:
        a.pods = a.steps * a.batch
    return a


# per-workload defaults; bytes = algorithmic bytes per node-eval
WORKLOADS = {
    "c3": dict(steps=20, warmup=2, batch=None, nodes=100_000, pods=1_000_000, bytes=60),
    "c2": dict(steps=9, warmup=2, batch=None, nodes=5000, pods=50_000, bytes=68),
    # C2 + the launch-kernel features (volumes, SelectorSpread, pod anti-affinity): 68 B per node-eval
    # of the row and its label / taint ids; the volume slots and counted pairs a pod reads come on top
    "c2x": dict(steps=5, warmup=1, batch=None, nodes=5000, pods=20_000, bytes=68),
    "c4": dict(steps=10, warmup=1, batch=512, nodes=1_000_000, pods=None, bytes=60),
    "c5": dict(steps=3, warmup=1, batch=0, nodes=20_000, pods=0, bytes=60),
}


class Dist:
    """torchrun environment: one process per GPU over RCCL, or (--one-device) every rank on
    device 0 over gloo, the rehearsal a 1-GPU box allows."""

    def __init__(self, a):
        import torch
        self.torch = torch
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.one = a.one_device
        self.dist = None
        if self.one:
            self.local = 0
            if self.world > 1:  # persistent kernels of all ranks must be co-resident on the one device
                os.environ.setdefault("KSIM_MAX_GRID", str(max(1, 256 // self.world // 2)))
        if self.world > 1:
            import torch.distributed as dist
            self.dist = dist
            if self.one:
                dist.init_process_group("gloo")
            else:
                torch.cuda.set_device(self.local)
                dist.init_process_group("nccl")

    def sync(self):
        self.torch.cuda.synchronize()
        if self.dist is not None:
            self.dist.barrier()
        self.torch.cuda.synchronize()

    def barrier(self):
        if self.dist is not None:
            self.dist.barrier()

    def allmax(self, x):
        if self.dist is None:
            return x
        t = self.torch.tensor([x], dtype=self.torch.float64, device="cpu" if self.one else "cuda")
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())

    def gather(self, obj):
        if self.dist is None:
            return [obj]
        out = [None] * self.world
        self.dist.all_gather_object(out, obj)
        return out

    def close(self):
        if self.dist is not None:
            self.dist.barrier()
            self.dist.destroy_process_group()


def timed_queue(a, D, make, steps, batch, pods):
    """Warm up on a separate scheduler (make()), then time `steps` calls of `batch` pods over the
    first `pods` pods of a fresh one, bracketed by barrier + device sync on every rank.
    Returns (placements, elapsed max over ranks, summed kernel ms, launches, last stats)."""
    import numpy as np
    w = make()
    first = 0
    for _ in range(a.warmup):
        D.barrier()
        w.schedule(first, min(batch, pods - first) if pods > first else 0)
        first = min(pods, first + batch)
    D.barrier()  # every rank's warmup kernels are done before any exchange buffer goes away
    w.close()
    g = make()
    outs, first, kms, launches, st = [], 0, 0.0, 0, None
    D.sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        cnt = min(batch, pods - first)
        if cnt <= 0:
            break
        o, _, st = g.schedule(first, cnt)
        outs.append(o)
        first += cnt
        kms += st.kernel_ms
        launches += st.kernel_launches
    D.sync()
    el = D.allmax(time.perf_counter() - t0)
    return g, np.concatenate(outs), el, kms, launches, st, first


class Local:
    """Timing bracket of a run that involves this rank only (no barrier, no cross-rank max)."""
    barrier = staticmethod(lambda: None)
    allmax = staticmethod(lambda x: x)

    @staticmethod
    def sync():
        import torch
        torch.cuda.synchronize()


def single_cluster(a, D, cl, preds, prios, mode, device):
    """One cluster per rank (N = 1: the headline; N > 1: the replica side line, or rank 0's
    single-GPU reference for the node-sharded run with D = Local)."""
    from ksim import scheduler
    make = lambda: scheduler.GenericScheduler(cl, preds, prios, device=device, mode=mode, collect_reasons=False)
    g, out, el, kms, launches, st, pods = timed_queue(a, D, make, a.steps, a.batch, a.pods)
    g.close()
    return dict(out=out, elapsed=el, kernel_ms=kms, launches=launches, mode=st.mode, blocks=st.blocks, pods=pods)


def node_sharded(a, D, cl, preds, prios):
    """One cluster, node-sharded over the D.world ranks: rank r holds
    name ranks [r*n/world, (r+1)*n/world); per pod the ranks exchange (fit count, max score,
    count at max) by device-initiated writes into each other's exchange buffers and reach the
    same selectHost decision.  Identical collective sequence on every rank, whatever fails."""
    import numpy as np
    from ksim import scheduler
    scheds = []

    def make():
        s = scheduler.ShardedScheduler(cl, preds, prios, D.rank, D.world, device=D.local)
        s.connect_torch(D.dist)
        scheds.append(s)
        return s

    err = None
    res = None
    try:
        g, out, el, kms, launches, st, pods = timed_queue(a, D, make, a.steps, a.batch, a.pods)
        res = dict(out=out, elapsed=el, kernel_ms=D.allmax(kms), launches=launches, mode=st.mode, blocks=st.blocks,
                   pods=pods, nodes_local=g.hi - g.lo)
    except Exception as e:  # noqa: BLE001 — reported in the JSON line
        err = "%s: %s" % (type(e).__name__, e)
    errs = D.gather(err)
    outs = D.gather(res["out"] if res else np.zeros(0, np.int32))
    for s in scheds:
        s.close()
    if any(errs):
        return {"error": [e for e in errs if e][0]}
    res["merged"] = scheduler.merge_sharded(outs)
    return res


def tree_mode(a, cl, preds, prios, device, ref):
    """The same queue through tree mode (KSIM_MODE_TREE, SURVEY.md §8f f4: incremental
    per-pod-class selection trees on one CU, O(classes x log N) per pod instead of the O(N)
    scan): pods/s over the same timed steps, and its placements against the scan's."""
    import numpy as np
    from ksim import abi, scheduler

    make = lambda: scheduler.GenericScheduler(cl, preds, prios, device=device, mode=abi.MODE_TREE, collect_reasons=False)
    g, out, el, kms, launches, st, pods = timed_queue(a, Local, make, a.steps, a.batch, a.pods)
    g.close()
    return {"value": round(pods / el, 1), "unit": "pods/s", "ms_per_step": round(el * 1e3 / a.steps, 4),
            "kernel_us_per_pod": round(kms * 1e3 / pods, 3),
            "mode": {3: "tree"}.get(st.mode, str(st.mode)),
            "parity_vs_scan": {"pods": int(len(out)), "match": bool(np.array_equal(out, ref[:len(out)]))},
            "note": "one wave on one CU per cluster; placements identical to the scan's; the headline "
                    "node-evals/s metric is defined on the full scan, so this is reported beside it"}


def cpu_baseline(a, cl, preds, prios, placements, unit="pods/s"):
    """The C port of the Go path (oracle/cpu_ref.c, OpenMP node-parallel like
    workqueue.Parallelize) on bounded prefixes of the same queue, at 1, 16 and all host threads;
    parity = its placements equal the GPU's over the largest prefix."""
    import numpy as np
    from ksim import scheduler
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref
    n = cl.n_nodes
    cfg = scheduler.make_config(preds, prios)
    avail = len(os.sched_getaffinity(0))
    legs = []
    # node-eval budgets: ~10 s per leg at the measured C3 rates (1 thread ~0.09e9, 16 threads
    # ~0.28e9 node-evals/s); the all-cores leg oversubscribes the box's CPU share, so it gets less
    for t, budget in ((1, 9e8), (min(a.cpu_threads, avail), 2.8e9), (min(avail, 64), 3e8)):
        if any(t == x[0] for x in legs):
            continue
        S = int(min(a.cpu_sample, len(placements), max(20, budget // n)))
        t1 = time.perf_counter()
        ref, _, _, _ = cpu_ref.run(cl, cfg, 0, S, threads=t)
        s = time.perf_counter() - t1
        legs.append((t, S, s, bool(np.array_equal(ref, placements[:S]))))
    main = max(legs, key=lambda x: (x[0] == min(a.cpu_threads, avail), x[1]))
    t, S, s, match = main
    cpu = {"value": round(S / s, 1), "unit": unit, "cores": t, "kind": "port",
           "sample": "first %d pods of the same %s queue on the same %d-node cluster (oracle/cpu_ref.c, "
                     "OpenMP node-parallel like workqueue.Parallelize), %.2f s" % (S, a.workload.upper(), n, s),
           "node_evals_per_s": round(S * n / s, 1),
           "by_threads": [{"cores": x[0], "pods": x[1], "seconds": round(x[2], 3), "value": round(x[1] / x[2], 1)}
                          for x in legs],
           "host_cpus_visible": avail}
    parity = {"prefix_pods": max(x[1] for x in legs), "match": all(x[3] for x in legs)}
    return cpu, parity


def cpu_baseline_objects(a, objs, preds, prios, placements, cl, budget_s=10.0):
    """C2x: the C port does not restate volumes / spread / affinity, so the CPU leg is the object
    oracle (oracle/ksim_ref.py, one thread, pure Python) on a prefix sized to ~budget_s; parity =
    its placements equal the GPU's over that prefix."""
    import numpy as np
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import ksim_ref as R
    listers = R.VolumeListers(objs["pvs"], objs["pvcs"])
    custom = {k: v for k, v in R.volume_predicates(listers).items() if k in preds}
    queue = objs["pods"]                            # scheduling order (the cluster's queue)
    S, s = 8, 0.0
    while True:
        t1 = time.perf_counter()
        want, _ = R.simulate(objs["nodes"], [], list(reversed(queue[:S])), set(preds), list(prios), custom,
                             spread=R.SpreadListers(services=objs["services"]))
        s = time.perf_counter() - t1
        if s >= budget_s / 4 or S >= min(a.cpu_sample, len(placements)):
            break
        S = min(int(S * max(2.0, budget_s / max(s, 1e-3))), min(a.cpu_sample, len(placements)))
    idx = {nm: i for i, nm in enumerate(cl.names)}
    ref = np.array([idx[h] if h is not None else -1 for _, h, _ in want], np.int32)
    cpu = {"value": round(S / s, 2), "unit": "pods/s", "cores": 1, "kind": "port",
           "sample": "first %d pods of the same C2x queue on the same %d-node cluster (oracle/ksim_ref.py, the "
                     "object-level restatement in pure Python: the C port does not cover volumes / spread / "
                     "affinity), %.2f s" % (S, cl.n_nodes, s),
           "node_evals_per_s": round(S * cl.n_nodes / s, 1)}
    return cpu, {"prefix_pods": S, "match": bool(np.array_equal(ref, placements[:S]))}


def main():
    a = parse()
    if a.workload == "c5":
        return main_c5(a)
    import numpy as np
    from ksim import abi, synth

    D = Dist(a)
    world, rank, local = D.world, D.rank, D.local
    W = WORKLOADS[a.workload]
    if a.workload == "c3":
        cl, preds, prios = synth.config_c3(a.nodes, a.pods)
        desc = "C3: %d nodes, %d-pod queue, default predicates + LeastRequested(1) + BalancedResourceAllocation(1)"
        data = "synthetic (splitmix64 seed 3, SURVEY.md §8d C3)"
    elif a.workload == "c4":
        cl, preds, prios = synth.config_c4(a.nodes, a.pods)
        desc = "C4: %d nodes, %d-pod queue, default predicates + LeastRequested(1) + BalancedResourceAllocation(1)"
        data = "synthetic (splitmix64 seed 4, SURVEY.md §8d C4)"
    elif a.workload == "c2x":
        cl, preds, prios, objs = synth.config_c2x(a.nodes, a.pods)
        desc = ("C2x: %d C2 nodes in zones, %d pods: C2's plus volumes (GCE PD / EBS / zoned PVCs), services "
                "(SelectorSpread), hostname anti-affinity; DefaultProvider")
        data = "synthetic (random.Random seed 6 objects through ingest; C2 extended with the launch-kernel features)"
    else:
        cl, preds, prios = synth.config_c2(a.nodes, a.pods)
        desc = ("C2: %d heterogeneous nodes (labels, taints, NotReady), %d pods with nodeSelector, host ports, "
                "tolerations, BestEffort; DefaultProvider")
        data = "synthetic (random.Random seed 2 objects through ingest, SURVEY.md §8d C2)"
    n = cl.n_nodes
    mode = {"auto": abi.MODE_AUTO, "launch": abi.MODE_LAUNCH, "persistent": abi.MODE_PERSISTENT, "tree": abi.MODE_TREE}[a.mode]
    sharded_head = world > 1 and a.shard == "nodes" and a.workload not in ("c2", "c2x")  # sharding: resource-only pods

    # ---- the one cluster: single GPU (N = 1), or node-sharded across the N ranks ----
    single = None
    if world == 1 or not sharded_head or rank == 0:
        # N = 1 headline; with N > 1 rank 0's single-GPU run is the sharded run's parity reference
        single = single_cluster(a, D if (world == 1 or not sharded_head) else Local, cl, preds, prios, mode, local)
    D.barrier()
    head = single
    sharded = None
    if sharded_head:
        sharded = node_sharded(a, D, cl, preds, prios)
        head = sharded
    replicas = None
    if world > 1 and a.shard != "none" and not (a.shard == "replicas" or a.workload in ("c2", "c2x")):
        # side line: each rank its own cluster under its own LeastRequested weight (weak scaling)
        prios_r = [(k, w + rank) if k == "LeastRequestedPriority" else (k, w) for k, w in prios]
        r_args = argparse.Namespace(**vars(a))
        r_args.pods = min(a.pods, a.replica_pods)
        r_args.batch = -(-r_args.pods // a.steps)
        rr = single_cluster(r_args, D, cl, preds, prios_r, mode, local)
        replicas = {"value": round(world * rr["pods"] / rr["elapsed"], 1), "unit": "pods/s", "scaling": "weak",
                    "ranks": world, "pods_per_rank": rr["pods"],
                    "ms_per_step": round(rr["elapsed"] * 1e3 / a.steps, 4),
                    "note": "every rank schedules its own %d-node cluster under LeastRequested weight 1 + rank "
                            "(a what-if sweep), no data-path collective" % n}
    if world > 1 and a.shard == "replicas":
        prios_r = [(k, w + rank) if k == "LeastRequestedPriority" else (k, w) for k, w in prios]
        head = single_cluster(a, D, cl, preds, prios_r, mode, local)

    tree = None
    if rank == 0 and a.tree and a.mode != "tree" and a.workload in ("c3", "c4") and single is not None:
        tree = tree_mode(a, cl, preds, prios, local, single["out"])
    cpu = parity = None
    if rank == 0 and a.cpu_sample > 0 and single is not None:
        if a.workload == "c2x":
            cpu, parity = cpu_baseline_objects(a, objs, preds, prios, single["out"], cl)
        else:
            cpu, parity = cpu_baseline(a, cl, preds, prios, single["out"])

    if rank == 0:
        if "error" in head:
            line = {"metric": "pods scheduled/sec + node-evals/sec at 100k nodes, 1/2/4/8 MI355X", "value": None,
                    "error": head["error"], "n_gpus": world}
            print(json.dumps(line))
            D.close()
            return
        pods_timed = head["pods"]
        elapsed = head["elapsed"]
        value = (world if (world > 1 and a.shard == "replicas") else 1) * pods_timed / elapsed
        mode_used = head["mode"]
        n_local = head.get("nodes_local", n)
        # dominant kernel: the scan (launch mode: one launch per pod) or the persistent kernel;
        # per-launch average from HIP events on the library's stream (max over ranks when sharded)
        if mode_used == abi.MODE_LAUNCH:
            pods_per_launch = 1
            avg_launch_s = head["kernel_ms"] / 1e3 / max(pods_timed, 1)
        else:
            pods_per_launch = a.batch
            avg_launch_s = head["kernel_ms"] / 1e3 / max(head["launches"], 1)
        achieved = W["bytes"] * n_local * min(pods_per_launch, pods_timed) / avg_launch_s / 1e9
        tree_kernel = mode_used == abi.MODE_TREE
        bound = int((head.get("merged", head["out"]) >= 0).sum())
        line = {
            "metric": ("pods scheduled/sec + node-evals/sec at 100k nodes, 1/2/4/8 MI355X" if a.workload == "c3" else
                       "pods scheduled/sec + node-evals/sec, %s (%d nodes)" % (a.workload.upper(), n)),
            "value": round(value, 1),
            "unit": "pods/s",
            "node_evals_per_s": round(value * n, 1),
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 4),
            "higher_is_better": True,
            "scaling": "strong" if sharded_head else "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": data,
            "config": {"workload": desc % (n, a.pods),
                       "nodes": n, "pods_timed": pods_timed, "pods_per_step": a.batch,
                       "timed_region": "the whole %d-pod queue from the empty cluster (warmup on a separate copy)"
                                       % pods_timed if pods_timed == a.pods else "the first %d pods" % pods_timed,
                       "global_batch": a.batch,
                       "mode": {1: "launch", 2: "persistent", 3: "tree"}.get(mode_used, str(mode_used)),
                       "blocks": head["blocks"],
                       "parallelism": ("node-sharded x%d" % world if sharded_head else
                                       "scenario-replicas x%d" % world if world > 1 else "single-gpu")},
            "roofline": {"bound": "hbm", "achieved": None if tree_kernel else round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": None if tree_kernel else round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None if (tree_kernel or world > 1) else
                         pmc_traffic(a.workload + ("" if mode_used == abi.MODE_PERSISTENT else "_launch"),
                                     n * pods_per_launch),
                         "traffic_unit": "GB per launch (PMC)", "bytes_per_node_eval": W["bytes"],
                         "nodes_per_gpu": n_local,
                         "avg_launch_us": round(avg_launch_s * 1e6, 3), "pods_per_launch": pods_per_launch,
                         **({"note": "tree mode reads O(classes x log N) bytes per pod, not the table: no HBM "
                                     "roofline applies"} if tree_kernel else {})},
            "cpu_baseline": cpu,
            "parity": parity,
            "pods_bound": bound,
        }
        if tree is not None:
            line["tree_mode"] = tree
        if sharded is not None:
            ns = {"ranks": world, "nodes_per_rank": n_local, "scaling": "strong",
                  "exchange": "device-initiated system-scope stores into every rank's fine-grained exchange buffer "
                              "(IPC)" + (", all ranks on device 0 (rehearsal)" if D.one else " over xGMI")}
            if single is not None:
                S = min(len(single["out"]), len(sharded["merged"]))
                ns["parity"] = {"pods": int(S), "vs": "single-GPU run of the same cluster and queue",
                                "match": bool(np.array_equal(sharded["merged"][:S], single["out"][:S]))}
                ns["single_gpu_value"] = round(single["pods"] / single["elapsed"], 1)
            line["node_sharded"] = ns
        if replicas is not None:
            line["replicas"] = replicas
        print(json.dumps(line))
    D.close()


def main_c5(a):
    """C5 (BASELINE.json configs[4]): the 4,096-scenario policy/weight sweep on a 20k-node
    cluster, scenario-parallel across ranks (rank r takes a contiguous share of the scenarios,
    no collective).  A step = one ksim_sweep call: every local scenario schedules the first
    --sweep-pods pods of the queue on its own copy of the snapshot (strong scaling: the total
    scenario count is fixed).  value = scenario-pods scheduled by all ranks per second."""
    import numpy as np
    import torch
    from ksim import scheduler, synth

    if a.sweep_form == "scan":
        os.environ["KSIM_SWEEP_SCAN"] = "1"
    D = Dist(a)
    world, rank, local = D.world, D.rank, D.local
    barrier_sync = D.sync

    cl, preds, scen = synth.config_c5(a.sweep_nodes, a.sweep_pods)
    scen = scen[:a.scenarios]
    lo, hi = rank * len(scen) // world, (rank + 1) * len(scen) // world
    mine = scen[lo:hi]
    g = scheduler.GenericScheduler(cl, preds, scen[0], device=local, collect_reasons=False)
    for _ in range(a.warmup):
        g.sweep(mine, 0, a.sweep_pods)
    barrier_sync()
    t0 = time.perf_counter()
    kernel_ms = 0.0
    for _ in range(a.steps):
        out, ctr, st = g.sweep(mine, 0, a.sweep_pods)
        kernel_ms += st.kernel_ms
    tree = st.mode == 3  # KSIM_MODE_TREE: one tree-mode wave per scenario (ksim_tree.hip)
    barrier_sync()
    elapsed = D.allmax(time.perf_counter() - t0)
    n = cl.n_nodes
    scen_pods = len(scen) * a.sweep_pods * a.steps
    value = scen_pods / elapsed
    avg_launch_s = kernel_ms / 1e3 / a.steps
    evals_per_launch = len(mine) * a.sweep_pods * n
    achieved = BYTES_PER_NODE_EVAL * evals_per_launch / avg_launch_s / 1e9
    cpu = parity = None
    if rank == 0 and a.cpu_sample > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cpu_ref
        threads = max(1, min(a.cpu_threads, len(os.sched_getaffinity(0))))
        S = min(a.cpu_sample, a.sweep_pods)
        t1 = time.perf_counter()
        ref, _, _, _ = cpu_ref.run(cl, scheduler.make_config(preds, mine[0]), 0, S, threads=threads)
        cpu_s = time.perf_counter() - t1
        cpu = {"value": round(S / cpu_s, 1), "unit": "scenario-pods/s", "cores": threads, "kind": "port",
               "sample": "scenario 0, first %d pods (oracle/cpu_ref.c, OpenMP node-parallel), %.1f s" % (S, cpu_s),
               "node_evals_per_s": round(S * n / cpu_s, 1)}
        parity = {"scenario": lo, "prefix_pods": S, "match": bool(np.array_equal(ref, out[0][:S]))}
    if rank == 0:
        line = {
            "metric": "scenario-pods scheduled/sec + node-evals/sec, 4,096-scenario policy sweep on 20k nodes (C5)",
            "value": round(value, 1),
            "unit": "scenario-pods/s",
            "node_evals_per_s": round(value * n, 1),
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed * 1e3 / a.steps, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64 (exact integer arithmetic below 2^48)",
            "data": "synthetic (splitmix64 seed 5, SURVEY.md \u00a78d C5)",
            "config": {"workload": "C5: %d scenarios (wLR 1..16 x wBRA 1..16 x wMR 0..15) x %d pods on %d nodes"
                                   % (len(scen), a.sweep_pods, n),
                       "nodes": n, "scenarios": len(scen), "scenarios_per_rank": len(mine),
                       "pods_per_scenario": a.sweep_pods, "parallelism": "scenario-parallel x%d" % world,
                       "form": "tree (one tree-mode wave per scenario)" if tree else "scan (one workgroup per scenario)"},
            "roofline": {"bound": "hbm", "achieved": None if tree else round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s",
                         "frac": None if tree else round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None if tree else pmc_traffic("c5", evals_per_launch),
                         "traffic_unit": "GB per launch (PMC)",
                         "bytes_per_node_eval": BYTES_PER_NODE_EVAL, "avg_launch_us": round(avg_launch_s * 1e6, 3),
                         "node_evals_per_launch": evals_per_launch,
                         **({"note": "tree form reads O(classes x log N) bytes per pod: achieved is the "
                                     "scan-equivalent rate"} if tree else {})},
            "cpu_baseline": cpu,
            "parity": parity,
        }
        print(json.dumps(line))
    D.close()


if __name__ == "__main__":
    main()
