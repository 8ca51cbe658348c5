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
    """HBM traffic of the dominant kernel from the PMC profile collected at this round's code
    (profiles/r6, r5, r4 or r3 /pmc_<workload>.json: FETCH_SIZE (x2, the gfx950 correction) + WRITE_SIZE per
    dispatch in separate rocprofv3 --pmc passes of the bench command, tools/gpu_pmc.sh +
    tools/pmc_summary.py, as MI355X_MICROARCH.md prescribes), scaled to this launch's node-evals;
    None when no such profile exists.  Returns {"gb_per_launch", "bytes_per_node_eval", "source"}."""
    path = None
    for rnd in ("r6", "r5", "r4", "r3"):  # the newest round's profile of this kernel
        path = os.path.join(ROOT, "profiles", rnd, "pmc_%s.json" % workload)
        if os.path.exists(path):
            break
    try:
        d = json.load(open(path))
        per_eval = float(d["hbm_bytes_per_node_eval"])
    except (OSError, KeyError, ValueError):
        return None
    return {"gb_per_launch": round(per_eval * evals_per_launch / 1e9, 6), "bytes_per_node_eval": round(per_eval, 4),
            "source": os.path.relpath(path, ROOT), "profiled": d.get("profiled")}


def roofline_bound(alg_bytes, traffic, launch_s=None, on_chip=False):
    """"hbm" when the kernel moves about the algorithmic bytes through HBM; "latency" when the PMC
    bytes per node-eval are far below them (the table is on chip: the per-pod exchange bounds it),
    or when the measured HBM traffic runs at under a tenth of the peak rate (what it moves is the
    exchange's polling, not the table).  Without a PMC file: "latency" for a persistent kernel
    whose rows live in LDS (on_chip), else "hbm"."""
    if traffic is None:
        return "latency" if on_chip else "hbm"
    if traffic["bytes_per_node_eval"] < 0.1 * alg_bytes:
        return "latency"
    if launch_s and traffic["gb_per_launch"] / launch_s < 0.1 * HBM_PEAK_GBS:
        return "latency"
    return "hbm"


def effective_cpus():
    """Host cores this process may use: the affinity mask, capped by a cgroup CPU quota and by the
    box's thread budget (OMP_NUM_THREADS / MAX_JOBS, 16 on the GPU box)."""
    n = len(os.sched_getaffinity(0))
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            f = open(path).read().split()
            if path.endswith("cpu.max"):
                if f[0] != "max":
                    n = min(n, max(1, int(f[0]) // int(f[1])))
            elif int(f[0]) > 0:
                per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                n = min(n, max(1, int(f[0]) // per))
        except (OSError, ValueError, IndexError):
            pass
    for k in ("OMP_NUM_THREADS", "MAX_JOBS"):
        v = os.environ.get(k, "")
        if v.isdigit() and int(v) > 0:
            n = min(n, int(v))
    return n


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
                    help="most pods in a CPU-baseline prefix (0 = skip); each leg is sized to ~8 s of CPU work")
    ap.add_argument("--c4-pods", type=int, default=20000,
                    help="c3 line: pods of the 1M-node C4 streaming side measurement (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--per-pod-calls", type=int, default=200,
                    help="c2 / c2x: timed ksim_k8s_cache_schedule calls through the C++ scheduler cache at each "
                         "cached-pod mark (0 = skip the per_pod side line)")
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


def cpu_baseline(a, cl, preds, prios, placements, unit="pods/s", leg_s=8.0, full_parity=False):
    """The C port of the Go path (oracle/cpu_ref.c: one OpenMP team per call splitting every pod's
    node loop, like workqueue.Parallelize(16)) over the same tables the device loads
    (scheduler.plan: class tables, affinity / spread / volume tables), on prefixes of the same
    queue at 1 and 16 threads (and every usable core when the box has more than 16), each leg
    sized to ~leg_s seconds from a short calibration run; parity = its placements equal the GPU's
    over every prefix.  full_parity: also run the whole queue at 16 threads when that fits ~30 s."""
    import numpy as np
    from ksim import scheduler
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref
    n = cl.n_nodes
    plan = scheduler.plan(cl, preds, prios)
    cores = effective_cpus()
    total = len(placements)

    def run(S, t):
        t1 = time.perf_counter()
        ref = cpu_ref.run(cl, None, 0, S, threads=t, plan=plan)[0]
        return time.perf_counter() - t1, bool(np.array_equal(ref, placements[:S]))

    legs = []
    for t in sorted({1, min(a.cpu_threads, cores), cores}):
        S0 = int(min(total, a.cpu_sample, max(8, 4e7 // n)))  # calibration: ~40M node-evals
        s0, ok0 = run(S0, t)
        S = int(min(total, a.cpu_sample, max(S0, S0 * leg_s / max(s0, 1e-3))))
        s, ok = run(S, t) if S > S0 else (s0, ok0)
        legs.append((t, S, s, ok and ok0))
    main = max(legs, key=lambda x: (x[0] == min(a.cpu_threads, cores), x[1]))
    t, S, s, match = main
    cpu = {"value": round(S / s, 1), "unit": unit, "cores": t, "kind": "port",
           "sample": "first %d pods of the same %s queue on the same %d-node cluster (oracle/cpu_ref.c over the "
                     "tables the device loads, one OpenMP team per call like workqueue.Parallelize), %.2f s"
                     % (S, a.workload.upper(), n, s),
           "node_evals_per_s": round(S * n / s, 1),
           "by_threads": [{"cores": x[0], "pods": x[1], "seconds": round(x[2], 3), "value": round(x[1] / x[2], 1)}
                          for x in legs],
           "host_cpus_visible": len(os.sched_getaffinity(0)), "host_cpus_usable": cores}
    parity = {"prefix_pods": max(x[1] for x in legs), "match": all(x[3] for x in legs)}
    if full_parity and parity["prefix_pods"] < total:
        t16 = min(a.cpu_threads, cores)
        rate = max(x[1] / x[2] for x in legs if x[0] == t16)
        if total / rate <= 30.0:
            s, ok = run(total, t16)
            parity = {"prefix_pods": total, "match": ok and parity["match"], "full_queue": True,
                      "seconds": round(s, 2), "cores": t16}
    return cpu, parity


def c4_stream_side(a):
    """BASELINE configs[3]'s node count on ONE GPU (1,000,000 nodes: 60 MB of table, beyond the
    per-CU LDS budget, so the fast kernel streams the rows from HBM): --c4-pods pods of the C4
    distributions, timed like the headline (warmup on a separate copy), with its own HBM roofline,
    PMC traffic and a parity prefix against the C port (16 threads)."""
    import numpy as np
    from ksim import abi, scheduler, synth
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import cpu_ref
    n, P = 1_000_000, a.c4_pods
    cl, preds, prios = synth.config_c4(n, P)
    steps = 10
    batch = -(-P // steps)
    a4 = argparse.Namespace(**vars(a))
    a4.warmup = 1
    make = lambda: scheduler.GenericScheduler(cl, preds, prios, device=0, collect_reasons=False)
    g, out, el, kms, launches, st, pods = timed_queue(a4, Local, make, steps, batch, P)
    g.close()
    avg = kms / 1e3 / max(launches, 1)
    achieved = 60 * n * batch / avg / 1e9
    traffic = pmc_traffic("c4", n * batch)
    S = min(P, 1500)
    t1 = time.perf_counter()
    ref = cpu_ref.run(cl, scheduler.make_config(preds, prios), 0, S, threads=min(a.cpu_threads, effective_cpus()))[0]
    cs = time.perf_counter() - t1
    return {"value": round(pods / el, 1), "unit": "pods/s", "node_evals_per_s": round(pods * n / el, 1),
            "config": "C4 node count on one GPU: %d nodes, %d pods of the C4 distributions, default predicates + "
                      "LeastRequested(1) + BalancedResourceAllocation(1), %d steps of %d pods" % (n, P, steps, batch),
            "mode": {1: "launch", 2: "persistent", 3: "tree"}.get(st.mode, str(st.mode)),
            "form": "streaming (rows from HBM)" if st.mode == abi.MODE_PERSISTENT else "other",
            "ms_per_step": round(el * 1e3 / steps, 4),
            "roofline": {"bound": roofline_bound(60, traffic), "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic and traffic["gb_per_launch"], "traffic_unit": "GB per launch (PMC)",
                         "traffic_source": traffic and traffic["source"], "bytes_per_node_eval": 60,
                         "avg_launch_us": round(avg * 1e6, 3), "pods_per_launch": batch},
            "cpu_baseline": {"value": round(S / cs, 1), "unit": "pods/s", "cores": min(a.cpu_threads, effective_cpus()),
                             "kind": "port", "sample": "first %d pods, oracle/cpu_ref.c, %.2f s" % (S, cs)},
            "parity": {"prefix_pods": S, "match": bool(np.array_equal(ref, out[:S]))}}


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
    # node sharding takes every workload's pods: Phase A (reduce-class maxima, inter-pod affinity
    # min / max, spread maxima and zone sums) is exchanged across the ranks
    sharded_head = world > 1 and a.shard == "nodes"

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
    if world > 1 and a.shard != "none" and a.shard != "replicas":
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
    c4 = None
    if world == 1 and a.workload == "c3" and a.c4_pods > 0 and a.mode == "auto":
        c4 = c4_stream_side(a)
    per_pod = None
    if world == 1 and a.workload in ("c2", "c2x") and a.per_pod_calls > 0:
        per_pod = per_pod_side(a)
    cpu = parity = None
    if rank == 0 and a.cpu_sample > 0 and single is not None:
        cpu, parity = cpu_baseline(a, cl, preds, prios, single["out"], full_parity=a.workload in ("c2", "c2x"))

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
        # the persistent kernels keep up to ~400k rows per device in LDS (ksim_pfast_config /
        # the general kernel's plan); beyond that the fast kernel streams rows from HBM
        on_chip = mode_used == abi.MODE_PERSISTENT and n_local <= 400_000
        bound = int((head.get("merged", head["out"]) >= 0).sum())
        traffic = None if (tree_kernel or world > 1) else \
            pmc_traffic(a.workload + ("" if mode_used == abi.MODE_PERSISTENT else "_launch"),
                        n * min(pods_per_launch, pods_timed))
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
            "roofline": {"bound": "latency" if tree_kernel else roofline_bound(W["bytes"], traffic, avg_launch_s, on_chip),
                         "achieved": None if tree_kernel else round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": None if tree_kernel else round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic and traffic["gb_per_launch"],
                         "traffic_unit": "GB per launch (PMC)",
                         "traffic_bytes_per_node_eval": traffic and traffic["bytes_per_node_eval"],
                         "traffic_source": traffic and traffic["source"],
                         "bytes_per_node_eval": W["bytes"],
                         "nodes_per_gpu": n_local,
                         "avg_launch_us": round(avg_launch_s * 1e6, 3), "pods_per_launch": pods_per_launch,
                         **({"note": "tree mode reads O(classes x log N) bytes per pod, not the table: no HBM "
                                     "roofline applies"} if tree_kernel else
                            {"note": "achieved = algorithmic bytes / launch time; the PMC traffic shows the table "
                                     "stays on chip (LDS), so the per-pod cross-CU exchange, not HBM, bounds it"}
                            if roofline_bound(W["bytes"], traffic, avg_launch_s, on_chip) == "latency" else {})},
            "cpu_baseline": cpu,
            "parity": parity,
            "pods_bound": bound,
        }
        if tree is not None:
            line["tree_mode"] = tree
        if c4 is not None:
            line["c4_stream"] = c4
        if per_pod is not None:
            line["per_pod"] = per_pod
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


def per_pod_side(a, marks=(1000, 20000)):
    """The per-pod drop-in's latency: genericScheduler.Schedule +
    assume as scheduleOne drives them (scheduler.go:431-484), through the C++ scheduler cache
    (ksim_k8s_cache_schedule, the call a cgo adapter makes: encode, incremental affinity / volume
    sync, one launch, one stream sync, results in host-mapped memory) — timed over
    `a.per_pod_calls` consecutive pods of the workload's queue once `m` pods are cached, for each
    mark m (the calls before a mark are the untimed fill).  The pods of a timed window are
    flattened to their C structs beforehand (a Go adapter's cost, not the library's); each call is
    timed on its own for the percentiles.  The cluster is the workload's nodes (and, for C2x, its
    PV / PVC listers and services)."""
    import ctypes as C
    from ksim import abi, synth
    from ksim.frontend import K8sCache, _Keep, lib as k8s_lib
    from ksim.spread import SpreadListers
    calls = a.per_pod_calls
    total = max(marks) + 2 * calls
    if a.workload == "c2x":
        nodes, pods, pvs, pvcs, services = synth.c2x_objects(a.nodes, total)
        kw = dict(pvs=pvs, pvcs=pvcs, spread=SpreadListers(services=services))
    else:
        nodes, pods = synth.c2_objects(a.nodes, total)
        kw = {}
    preds, prios = scheduler_provider()
    sc = K8sCache(preds, prios, **kw)
    L = k8s_lib()
    t_start = time.perf_counter()
    try:
        for nd in nodes:
            sc.add_node(nd)
        out, i, bound = [], 0, 0
        for m in marks:
            while i < m:
                bound += sc.schedule_one(pods[i])[0] is not None
                i += 1
                if i % 1000 == 0:
                    print("per_pod: %d pods cached (%.1f s)" % (i, time.perf_counter() - t_start), file=sys.stderr,
                          flush=True)
            keep = [_Keep() for _ in range(calls)]
            flat = [sc._pod(keep[j], pods[i + j]) for j in range(calls)]
            res = abi.Result()
            r0 = sc.stats()
            lat = []
            t0 = time.perf_counter()
            for j in range(calls):
                c0 = time.perf_counter()
                rc = L.ksim_k8s_cache_schedule(sc.h, flat[j], abi.SCHEDULE_ASSUME, C.byref(res))
                lat.append(time.perf_counter() - c0)
                if rc:
                    raise sc._err(rc, L.ksim_k8s_cache_last_error(sc.h))
                bound += res.node >= 0
            dt = time.perf_counter() - t0
            i += calls
            r1 = sc.stats()
            lat.sort()
            pct = lambda lt, q: round(lt[min(len(lt) - 1, int(q * len(lt)))] * 1e6, 1)
            # the Go adapter's pattern: Schedule with KSIM_SCHEDULE_ONLY, then the
            # pod, its spec.nodeName set to the host, through ksim_k8s_cache_assume_pod — two native
            # calls per pod (the next `calls` pods of the queue)
            keep2 = [_Keep() for _ in range(calls)]
            flat2 = [sc._pod(keep2[j], pods[i + j]) for j in range(calls)]
            names = [C.c_char_p(n.encode()) for n in sc.names]
            lat2 = []
            t1 = time.perf_counter()
            for j in range(calls):
                c0 = time.perf_counter()
                rc = L.ksim_k8s_cache_schedule(sc.h, flat2[j], abi.SCHEDULE_ONLY, C.byref(res))
                if rc:
                    raise sc._err(rc, L.ksim_k8s_cache_last_error(sc.h))
                if res.node >= 0:
                    flat2[j]._obj.node_name = names[res.node]
                    rc = L.ksim_k8s_cache_assume_pod(sc.h, flat2[j])
                    if rc:
                        raise sc._err(rc, L.ksim_k8s_cache_last_error(sc.h))
                    bound += 1
                lat2.append(time.perf_counter() - c0)
            dt2 = time.perf_counter() - t1
            i += calls
            lat2.sort()
            out.append({"cached_pods": m, "calls": calls, "us_per_call": round(dt / calls * 1e6, 1),
                        "p50_us": pct(lat, 0.5), "p90_us": pct(lat, 0.9), "p99_us": pct(lat, 0.99),
                        "affinity_table_loads": r1[0] - r0[0], "volume_table_loads": r1[1] - r0[1],
                        "volume_table_grows": r1[2] - r0[2],
                        "adapter_pattern": {"calls": "ksim_k8s_cache_schedule(SCHEDULE_ONLY) + ksim_k8s_cache_assume_pod",
                                            "us_per_pod": round(dt2 / calls * 1e6, 1), "p50_us": pct(lat2, 0.5),
                                            "p99_us": pct(lat2, 0.99)}})
        st = sc.stats()
        return {"front_end": "C++ ksim_k8s_cache_schedule (SCHEDULE_ASSUME)", "marks": out, "pods_bound": bound,
                "nodes": len(nodes), "affinity_table_loads": st[0], "volume_table_loads": st[1],
                "volume_table_grows": st[2], "class_table_loads": st[3],
                "note": "wall time per scheduleOne-equivalent native call (encode + table sync + one launch "
                        "+ one sync + assume), pods of the same workload queue in order"}
    finally:
        sc.close()


def scheduler_provider():
    from ksim import scheduler
    return scheduler.provider("DefaultProvider")


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
        threads = max(1, min(a.cpu_threads, effective_cpus()))
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
            "roofline": {"bound": "latency" if tree else "hbm", "achieved": None if tree else round(achieved, 1),
                         "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": None if tree else round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": None if tree else (pmc_traffic("c5", evals_per_launch) or {}).get("gb_per_launch"),
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
