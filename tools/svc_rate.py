"""Throughput of a batch with CheckServiceAffinity lenders (services selecting the pods), launch
form against the general persistent kernel, on one GPU.
Usage (GPU box, repo root): python3 tools/svc_rate.py [n_nodes] [n_pods]"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "kubernetes-schedule-simulator_amd"))
sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "tests"))
from ksim import abi, ingest, scheduler, spread  # noqa: E402
from workloads import rnd_svc_affinity_workload  # noqa: E402

n_nodes = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
n_pods = int(sys.argv[2]) if len(sys.argv) > 2 else 5000
aff_labels = ["region", "rack"]
preds = ["GeneralPredicates", "PodToleratesNodeTaints", "CheckServiceAffinity"]
prios = [("LeastRequestedPriority", 1), ("BalancedResourceAllocation", 1)]
nodes, running, pods, services = rnd_svc_affinity_workload(7, n_nodes=n_nodes, n_pods=n_pods, full_labels=True)
order = list(reversed(pods))
cl = ingest.Cluster.from_objects(nodes, running, order, spread=spread.SpreadListers(services=services),
                                 service_affinity=aff_labels)
outs = {}
for mode in (abi.MODE_LAUNCH, abi.MODE_PERSISTENT):
    best = None
    for rep in range(3):
        g = scheduler.GenericScheduler(cl, preds, prios, mode=mode, service_affinity=aff_labels)
        try:
            t0 = time.perf_counter()
            out, _, st = g.schedule()
            dt = time.perf_counter() - t0
        finally:
            g.close()
        best = dt if best is None else min(best, dt)
    outs[mode] = out
    print("mode %d (ran %d): %d nodes x %d pods: %.1f ms, %.0f pods/s, %d bound" % (
        mode, st.mode, n_nodes, len(order), best * 1e3, len(order) / best, int((out >= 0).sum())), flush=True)
assert (outs[abi.MODE_LAUNCH] == outs[abi.MODE_PERSISTENT]).all()
print("placements identical")
