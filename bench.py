"""Benchmark of the MI355X per-pod scheduling cycle on BASELINE.json's headline workload.

Workload (BASELINE.json configs[2], SURVEY.md §8d "C3", the default; --workload c2 / c4 / c5
run the other configs the same way): 100,000 nodes, 1,000,000 mixed-size
pods, default predicates + LeastRequested(1) + BalancedResourceAllocation(1).  A "step" is
one ksim_schedule() call over the next `--batch` pods of the queue (each pod: predicates on
every node, priorities, selectHost, commit — strictly one after another), with the node
table and pod queue already resident in HBM.

N GPUs (torchrun, one process per GPU), two measurements in one run:
  * headline `value` (--shard replicas, default): scenario-parallel replicas — every rank runs
    its own 100k-node cluster with its own policy weights (a what-if sweep), no
    data-path collective; scaling "weak".  value = pods scheduled by all ranks / max time.
  * `node_sharded`: ONE 100k-node cluster split into N contiguous name-rank shards, one per
    GPU, each pod decided jointly through the per-pod exchange over xGMI (ksim_shard_*);
    pods/s of that one cluster (strong scaling), its placements checked against the
    single-cluster run of rank 0.  With --shard nodes this is the headline instead.

The JSON line also carries the roofline of the dominant kernel (algorithmic bytes per launch
÷ HIP-event launch duration, against the 8 TB/s HBM peak) and a cpu_baseline: the C oracle
(oracle/cpu_ref.c, a port of the Go path) timed on a bounded prefix of the same queue, whose
placements must equal the GPU's for the same prefix (reported as "parity").
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
    ap.add_argument("--steps", type=int, default=None, help="default: c3 100, c2 9, c4 10, c5 3")
    ap.add_argument("--warmup", type=int, default=None, help="default: c3 3, c2 2, c4 1, c5 1")
    ap.add_argument("--batch", type=int, default=None, help="pods per step (default: c3/c2 4096, c4 512)")
    ap.add_argument("--nodes", type=int, default=None, help="default: c3 100,000, c2 5,000, c4 1,000,000")
    ap.add_argument("--pods", type=int, default=None, help="queue length (default: c3 1M, c2 50k, c4 as needed)")
    ap.add_argument("--mode", default="auto", choices=["auto", "launch", "persistent", "tree"])
    ap.add_argument("--no-tree", dest="tree", action="store_false",
                    help="skip the tree-mode line measured beside the scan (c3/c4)")
    ap.add_argument("--cpu-sample", type=int, default=3000, help="pods in the CPU-baseline prefix (0 = skip)")
    ap.add_argument("--cpu-threads", type=int, default=16)
    ap.add_argument("--workload", default="c3", choices=["c3", "c2", "c4", "c5"],
                    help="c3: the headline metric (default); c2: 5k heterogeneous nodes with selectors, "
                         "ports and taints; c4: 1M nodes; c5: the 4,096-scenario policy sweep")
    ap.add_argument("--scenarios", type=int, default=4096, help="c5: total scenarios (split across ranks)")
    ap.add_argument("--sweep-nodes", type=int, default=20_000, help="c5: nodes per scenario")
    ap.add_argument("--sweep-form", default="auto", choices=["auto", "scan"],
                    help="c5: auto = tree form when eligible; scan = the per-scenario scan kernel")
    ap.add_argument("--sweep-pods", type=int, default=5000, help="c5: pods scheduled in every scenario")
    ap.add_argument("--shard", default="replicas", choices=["replicas", "nodes", "none"],
                    help="N>1 headline: replicas (weak) or one node-sharded cluster (strong); "
                         "the other one is measured as well unless 'none'")
    ap.add_argument("--shard-steps", type=int, default=20, help="timed steps of the node-sharded measurement")
    ap.add_argument("--one-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on device 0 (gloo), grids split so the "
                         "ranks' persistent kernels are co-resident")
    a = ap.parse_args()
    d = WORKLOADS[a.workload]
    for k in ("steps", "warmup", "batch", "nodes", "pods"):
        if getattr(a, k) is None:
            setattr(a, k, d.get(k))
    if a.pods is None:
        a.pods = (a.warmup + max(a.steps, a.shard_steps)) * a.batch
    return a


# per-workload defaults; bytes = algorithmic bytes per node-eval
WORKLOADS = {
    "c3": dict(steps=100, warmup=3, batch=4096, nodes=100_000, pods=1_000_000, bytes=60),
    "c2": dict(steps=9, warmup=2, batch=4096, nodes=5000, pods=50_000, bytes=68),
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


def node_sharded(a, D, cl, preds, prios, ref):
    """One cluster, node-sharded over the D.world ranks: rank r holds
    name ranks [r*n/world, (r+1)*n/world); per pod the ranks exchange (fit count, max score,
    count at max) by device-initiated writes into each other's exchange buffers and reach the
    same selectHost decision.  Returns the measurement dict (identical collective sequence on
    every rank, whatever fails)."""
    import numpy as np
    from ksim import scheduler
    out, err, s = np.zeros(0, np.int32), None, None
    try:
        s = scheduler.ShardedScheduler(cl, preds, prios, D.rank, D.world, device=D.local)
        s.connect_torch(D.dist)
    except Exception as e:  # noqa: BLE001 — reported in the JSON line
        err = "setup: %s" % e
    errs = D.gather(err)
    if any(errs):
        return {"error": [e for e in errs if e][0]}
    outs, first, kms, el = [], 0, 0.0, 0.0
    try:
        for _ in range(a.warmup):
            outs.append(s.schedule(first, a.batch)[0])
            first += a.batch
        D.sync()
        t0 = time.perf_counter()
        for _ in range(a.shard_steps):
            o, _, st = s.schedule(first, a.batch)
            outs.append(o)
            first += a.batch
            kms += st.kernel_ms
        D.sync()
        el = time.perf_counter() - t0
        out = np.concatenate(outs)
    except Exception as e:  # noqa: BLE001
        err = "schedule: %s" % e
    errs = D.gather(err)
    el = D.allmax(el)
    kms = D.allmax(kms)
    allouts = D.gather(out)
    s.close()
    if any(errs):
        return {"error": [e for e in errs if e][0]}
    merged = scheduler.merge_sharded(allouts)
    pods = a.shard_steps * a.batch
    res = {"value": round(pods / el, 1), "unit": "pods/s", "node_evals_per_s": round(pods * cl.n_nodes / el, 1),
           "scaling": "strong", "ranks": D.world, "nodes": cl.n_nodes, "nodes_per_rank": cl.n_nodes // D.world,
           "steps": a.shard_steps, "pods_per_step": a.batch, "ms_per_step": round(el * 1e3 / a.shard_steps, 4),
           "avg_launch_us": round(kms * 1e3 / a.shard_steps, 3),
           "exchange": "device-initiated system-scope stores into every rank's fine-grained exchange buffer (IPC)"
                       + (", all ranks on device 0 (rehearsal)" if D.one else " over xGMI")}
    if ref is not None:
        S = min(len(ref), len(merged))
        res["parity"] = {"pods": S, "vs": "single-GPU run of the same cluster and queue",
                         "match": bool(np.array_equal(merged[:S], ref[:S]))}
    return res


def tree_mode(a, cl, preds, prios, device, ref):
    """The same queue through tree mode (KSIM_MODE_TREE, SURVEY.md §8f f4: incremental
    per-pod-class selection trees on one CU, O(classes x log N) per pod instead of the O(N)
    scan): pods/s over the same timed steps, and its placements against the scan's."""
    import numpy as np
    from ksim import abi, scheduler
    g = scheduler.GenericScheduler(cl, preds, prios, device=device, mode=abi.MODE_TREE, collect_reasons=False)
    outs, first = [], 0
    for _ in range(a.warmup):
        outs.append(g.schedule(first, a.batch)[0])
        first += a.batch
    kms, mode_used = 0.0, 0
    t0 = time.perf_counter()
    for _ in range(a.steps):
        o, _, st = g.schedule(first, a.batch)
        outs.append(o)
        first += a.batch
        kms += st.kernel_ms
        mode_used = st.mode
    el = time.perf_counter() - t0
    out = np.concatenate(outs)
    pods = a.steps * a.batch
    return {"value": round(pods / el, 1), "unit": "pods/s", "ms_per_step": round(el * 1e3 / a.steps, 4),
            "kernel_us_per_pod": round(kms * 1e3 / pods, 3),
            "mode": {3: "tree"}.get(mode_used, str(mode_used)),
            "parity_vs_scan": {"pods": int(len(out)), "match": bool(np.array_equal(out, ref[:len(out)]))},
            "note": "one wave on one CU per cluster; placements identical to the scan's; the headline "
                    "node-evals/s metric is defined on the full scan, so this is reported beside it"}


def main():
    a = parse()
    if a.workload == "c5":
        return main_c5(a)
    import numpy as np
    import torch
    from ksim import abi, scheduler, synth

    D = Dist(a)
    world, rank, local, dist = D.world, D.rank, D.local, D.dist
    barrier_sync = D.sync

    total_pods = (a.warmup + a.steps) * a.batch
    if total_pods > a.pods:
        raise SystemExit("warmup+steps x batch = %d exceeds the %d-pod queue" % (total_pods, a.pods))
    W = WORKLOADS[a.workload]
    if a.workload == "c3":
        cl, preds, prios = synth.config_c3(a.nodes, a.pods)
        desc = "C3: %d nodes, %d-pod queue, default predicates + LeastRequested(1) + BalancedResourceAllocation(1)"
        data = "synthetic (splitmix64 seed 3, SURVEY.md §8d C3)"
    elif a.workload == "c4":
        cl, preds, prios = synth.config_c4(a.nodes, a.pods)
        desc = "C4: %d nodes, %d-pod queue, default predicates + LeastRequested(1) + BalancedResourceAllocation(1)"
        data = "synthetic (splitmix64 seed 4, SURVEY.md §8d C4)"
    else:
        cl, preds, prios = synth.config_c2(a.nodes, a.pods)
        desc = ("C2: %d heterogeneous nodes (labels, taints, NotReady), %d pods with nodeSelector, host ports, "
                "tolerations, BestEffort; DefaultProvider")
        data = "synthetic (random.Random seed 2 objects through ingest, SURVEY.md §8d C2)"
    prios0 = list(prios)  # the one cluster's policy (rank 0's replica, the node-sharded run)
    if rank > 0:  # what-if sweep: each replica scores with its own LeastRequested weight
        prios = [(k, w + rank) if k == "LeastRequestedPriority" else (k, w) for k, w in prios0]
    mode = {"auto": abi.MODE_AUTO, "launch": abi.MODE_LAUNCH, "persistent": abi.MODE_PERSISTENT, "tree": abi.MODE_TREE}[a.mode]
    g = scheduler.GenericScheduler(cl, preds, prios, device=local, mode=mode, collect_reasons=False)

    placements = []
    first = 0
    for _ in range(a.warmup):
        out, _, _ = g.schedule(first, a.batch)
        placements.append(out)
        first += a.batch
    barrier_sync()
    t0 = time.perf_counter()
    kernel_ms = 0.0
    launches = 0
    mode_used = blocks = 0
    for _ in range(a.steps):
        out, _, st = g.schedule(first, a.batch)
        placements.append(out)
        first += a.batch
        kernel_ms += st.kernel_ms
        launches += st.kernel_launches
        mode_used, blocks = st.mode, st.blocks
    barrier_sync()
    elapsed = D.allmax(time.perf_counter() - t0)
    placements = np.concatenate(placements)
    bound = int((placements >= 0).sum())

    pods_timed = a.steps * a.batch
    value = world * pods_timed / elapsed
    sharded = None
    if world > 1 and a.shard != "none" and a.workload != "c2":  # sharding takes resource-only pods
        sharded = node_sharded(a, D, cl, preds, prios0, placements if rank == 0 else None)
    n = cl.n_nodes
    # dominant kernel: the scan (launch mode: one launch per pod) or the persistent kernel
    if mode_used == abi.MODE_LAUNCH:
        pods_per_launch = 1
        avg_launch_s = kernel_ms / 1e3 / max(pods_timed, 1)
    else:
        pods_per_launch = a.batch
        avg_launch_s = kernel_ms / 1e3 / max(launches, 1)
    achieved = W["bytes"] * n * pods_per_launch / avg_launch_s / 1e9

    tree = None
    if rank == 0 and a.tree and a.mode != "tree" and a.workload in ("c3", "c4"):
        tree = tree_mode(a, cl, preds, prios, local, placements)

    cpu = None
    parity = None
    if rank == 0 and a.cpu_sample > 0:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import cpu_ref
        S = min(a.cpu_sample, len(placements), max(50, int(3e8 // n)))  # ~10-30 s of CPU work at most
        threads = max(1, min(a.cpu_threads, len(os.sched_getaffinity(0))))
        cfg = scheduler.make_config(preds, prios)
        t1 = time.perf_counter()
        ref_out, _, _, _ = cpu_ref.run(cl, cfg, 0, S, threads=threads)
        cpu_s = time.perf_counter() - t1
        cpu = {"value": round(S / cpu_s, 1), "unit": "pods/s", "cores": threads, "kind": "port",
               "sample": "first %d pods of the same %s queue on the same %d-node cluster (oracle/cpu_ref.c, "
                         "OpenMP node-parallel like workqueue.Parallelize), %.1f s" % (S, a.workload.upper(), n, cpu_s),
               "node_evals_per_s": round(S * n / cpu_s, 1)}
        parity = {"prefix_pods": S, "match": bool(np.array_equal(ref_out, placements[:S]))}

    if rank == 0:
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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": data,
            "config": {"workload": desc % (n, a.pods),
                       "nodes": n, "pods_per_step": a.batch, "global_batch": a.batch * world,
                       "mode": {1: "launch", 2: "persistent", 3: "tree"}.get(mode_used, str(mode_used)), "blocks": blocks,
                       "parallelism": "scenario-replicas x%d" % world if world > 1 else "single-gpu"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic(a.workload + ("" if mode_used == abi.MODE_PERSISTENT else "_launch"),
                                                n * pods_per_launch),
                         "traffic_unit": "GB per launch (PMC)", "bytes_per_node_eval": W["bytes"],
                         "avg_launch_us": round(avg_launch_s * 1e6, 3), "pods_per_launch": pods_per_launch,
                         **({"note": "tree mode reads O(classes x log N) bytes per pod: achieved is the scan-equivalent "
                                     "rate, not HBM traffic"} if mode_used == abi.MODE_TREE else {})},
            "cpu_baseline": cpu,
            "parity": parity,
            "pods_bound": bound,
        }
        if tree is not None:
            line["tree_mode"] = tree
        if sharded is not None:
            line["node_sharded"] = sharded
            if a.shard == "nodes" and "value" in sharded:  # the one node-sharded cluster as the headline
                line["replicas"] = {"value": line["value"], "scaling": "weak", "ms_per_step": line["ms_per_step"]}
                line.update(value=sharded["value"], node_evals_per_s=sharded["node_evals_per_s"], scaling="strong",
                            steps=a.shard_steps, ms_per_step=sharded["ms_per_step"])
                line["config"].update(parallelism="node-sharded x%d" % world, global_batch=a.batch)
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
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
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
