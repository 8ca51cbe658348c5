"""Diagnostic: the per-pod call through the C++ scheduler cache (bench.py's per_pod line), short
enough to run under rocprofv3 --kernel-trace --stats: fill `--fill` pods, then time `--calls`
ksim_k8s_cache_schedule calls (SCHEDULE_ASSUME) and print the wall-time percentiles."""
import argparse
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "kubernetes-schedule-simulator_amd"))
from ksim import abi, scheduler, synth  # noqa: E402
from ksim.frontend import K8sCache, _Keep, lib as k8s_lib  # noqa: E402
from ksim.spread import SpreadListers  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--workload", default="c2", choices=["c2", "c2x"])
ap.add_argument("--nodes", type=int, default=5000)
ap.add_argument("--fill", type=int, default=1000)
ap.add_argument("--calls", type=int, default=300)
a = ap.parse_args()
total = a.fill + a.calls
if a.workload == "c2x":
    nodes, pods, pvs, pvcs, services = synth.c2x_objects(a.nodes, total)
    kw = dict(pvs=pvs, pvcs=pvcs, spread=SpreadListers(services=services))
else:
    nodes, pods = synth.c2_objects(a.nodes, total)
    kw = {}
preds, prios = scheduler.provider("DefaultProvider")
sc = K8sCache(preds, prios, **kw)
L = k8s_lib()
for nd in nodes:
    sc.add_node(nd)
for i in range(a.fill):
    sc.schedule_one(pods[i])
keep = [_Keep() for _ in range(a.calls)]
flat = [sc._pod(keep[j], pods[a.fill + j]) for j in range(a.calls)]
res = abi.Result()
lat = []
s0 = sc.stats()
for j in range(a.calls):
    t0 = time.perf_counter()
    rc = L.ksim_k8s_cache_schedule(sc.h, flat[j], abi.SCHEDULE_ASSUME, C.byref(res))
    lat.append(time.perf_counter() - t0)
    assert rc == 0, rc
s1 = sc.stats()
lat.sort()
q = lambda f: lat[min(len(lat) - 1, int(f * len(lat)))] * 1e6
print("%s per-pod: mean %.1f us, p50 %.1f, p90 %.1f, p99 %.1f; table work (aff, vol loads, vol grows, class loads) %s"
      % (a.workload, sum(lat) / len(lat) * 1e6, q(0.5), q(0.9), q(0.99), [y - x for x, y in zip(s0, s1)]))
sc.close()
