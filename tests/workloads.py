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
