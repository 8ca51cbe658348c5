"""Seeded informer-style event streams for the per-pod drop-in tests: node add / update / remove,
pod add (bound elsewhere, or confirming an assumed pod) / update / remove, interleaved with
scheduleOne calls.  Events are generated against a shadow of the object-level oracle's cache so
every event is valid in the reference (cache.go would accept it)."""
import copy
import random

from workloads import rnd_nodes, rnd_pod


def event_stream(seed, ref, n_events=400, n_nodes=16, features=True, forget=0.0):
    """Yields (kind, payload) with kind in: add_node, update_node, remove_node, add_pod,
    update_pod, remove_pod, schedule.  The consumer applies each event to the oracle cache
    `ref` (ksim_ref.SchedulerCache) before pulling the next one; the generator reads it to pick
    valid targets."""
    rng = random.Random(seed)
    pool = rnd_nodes(rng, n_nodes + n_nodes // 2, features, name_fmt="node-{i}")
    listed, spare = pool[:n_nodes], pool[n_nodes:]
    for node in listed:
        yield "add_node", node
    k = 0
    for _ in range(n_events):
        names = list(ref.listed)
        added = [key for key in ref.pod_states if key not in ref.assumed]
        assumed = sorted(ref.assumed)
        if forget and assumed and rng.random() < forget:
            yield "forget_pod", copy.deepcopy(ref.pod_states[rng.choice(assumed)])
            continue
        r = rng.random()
        k += 1
        if r < 0.55 or not names:
            yield "schedule", rnd_pod(rng, "p-%d" % k, features)
        elif r < 0.63:
            p = rnd_pod(rng, "bound-%d" % k, features)
            p["spec"]["nodeName"] = rng.choice(names + ["gone-node"])
            yield "add_pod", p
        elif r < 0.71 and assumed:
            # the binding's watch event confirms the assumed pod, sometimes on another node
            p = copy.deepcopy(ref.pod_states[rng.choice(assumed)])
            if rng.random() < 0.15 and names:
                p["spec"]["nodeName"] = rng.choice(names)
            yield "add_pod", p
        elif r < 0.79 and added:
            yield "remove_pod", copy.deepcopy(ref.pod_states[rng.choice(sorted(added))])
        elif r < 0.83 and added:
            old = ref.pod_states[rng.choice(sorted(added))]
            new = copy.deepcopy(old)
            new["spec"]["containers"] = [{"resources": {"requests": {"cpu": rng.choice(["50m", "300m", "1"]),
                                                                     "memory": rng.choice(["64Mi", "1Gi"])}}}]
            yield "update_pod", (copy.deepcopy(old), new)
        elif r < 0.88 and spare:
            node = spare.pop(rng.randrange(len(spare)))
            yield "add_node", node
        elif r < 0.94:
            name = rng.choice(names)
            old = ref.nodes[name].node
            new = copy.deepcopy(old)
            q = rng.random()
            if q < 0.3:
                new["status"]["allocatable"]["cpu"] = "%dm" % rng.choice([500, 1000, 3000, 6000])
            elif q < 0.5:
                new["metadata"]["labels"] = {"tier": rng.choice("abcd"), "disk": rng.choice(["ssd", "hdd", "nvme"])}
            elif q < 0.65:
                new["spec"]["taints"] = rng.choice([[], [{"key": "dedicated", "value": "gpu", "effect": "NoSchedule"}],
                                                    [{"key": "spot", "value": "true", "effect": "PreferNoSchedule"}]])
            elif q < 0.8:
                # a node update without the pressure condition keeps the last status (SetNode)
                new["status"]["conditions"] = [c for c in new["status"]["conditions"] if c["type"] == "Ready"]
                if rng.random() < 0.5:
                    new["status"]["conditions"].append({"type": "MemoryPressure", "status": rng.choice(["True", "False"])})
            else:
                new["spec"]["unschedulable"] = not new["spec"].get("unschedulable", False)
            yield "update_node", (old, new)
        elif names:
            name = rng.choice(names)
            node = ref.nodes[name].node
            spare.append(copy.deepcopy(node))
            yield "remove_node", node
        else:
            yield "schedule", rnd_pod(rng, "p-%d" % k, features)


def apply(cache, ev):
    """Apply one event to a cache with the reference's method surface (ksim_ref.SchedulerCache
    or ksim.cache.SchedulerCache); schedule events return (host, FitError message)."""
    kind, x = ev
    if kind == "schedule":
        try:
            return cache.schedule_one(x)
        except Exception as e:  # ErrNoNodesAvailable (generic_scheduler.go:64) on both sides
            if "no nodes available to schedule pods" in str(e):
                return None, "no nodes available to schedule pods"
            raise
    if kind in ("update_node", "update_pod"):
        getattr(cache, kind)(*x)
    else:
        getattr(cache, kind)(x)
    return None
