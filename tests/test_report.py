"""The simulator's I/O around the scheduling path: the --podspec file (cmd/app/options/options.go:
73-99), the offline checkpoint (pkg/main.go:134-179), the Status the simulator leaves
(pkg/scheduler/simulator.go:108-213), GetReport (pkg/framework/report.go:96-174) and
ClusterCapacityReviewPrint (:176-237).

Fixtures: tests/golden/etc_pod.yaml is the reference's etc/pod.yaml; readme_failed_pods.txt is the
"Failed Pods" half of the sample output in the reference README (the "Successful Pods" half has
host names edited after rendering — its column is wider than any cell — so it is not a
rendering of any input and is not used).  CPU tests build the report from the oracle's scheduling
outcomes; the GPU tests check that the HIP path's report is byte-identical."""
import io
import json
import os
import re
from contextlib import redirect_stdout

import pytest

import ksim_ref as ref
from ksim import abi, cli, report, scheduler

GOLD = os.path.join(os.path.dirname(__file__), "golden")
PROVIDER = "DefaultProvider"


def _nodes(n, cpu="4", mem="8Gi", pods="110"):
    return [{"metadata": {"name": "node-%d" % i, "labels": {"kubernetes.io/hostname": "node-%d" % i}},
             "status": {"allocatable": {"cpu": cpu, "memory": mem, "pods": pods},
                        "conditions": [{"type": "Ready", "status": "True"}]}} for i in range(n)]


def _podspec():
    return scheduler.load_podspec(os.path.join(GOLD, "etc_pod.yaml"))


def _oracle_report(nodes, running, sim):
    keys, prios = ref.provider(PROVIDER)
    out, _ = ref.simulate(nodes, running, sim, keys, prios)
    order = list(reversed(sim))
    assert [o[0] for o in out] == [p["metadata"]["name"] for p in order]
    st = report.simulation_status(order, running, [(h, m) for _, h, m in out])
    return report.get_report(st)


# ----------------------------------------------------------------------------- podspec
def test_podspec_expansion_matches_parse_simulation_pod():
    spec = _podspec()
    assert [(s["name"], s["num"]) for s in spec] == [("A", 10), ("B", 10)]
    pods = scheduler.expand_simulation_pods(spec, "ns1")
    assert len(pods) == 20
    assert [p["metadata"]["name"] for p in pods[:2]] == ["A-0", "A-1"]
    for p in pods:
        m = p["metadata"]
        assert m["uid"] == m["name"] and m["namespace"] == "ns1"
        assert m["labels"] == {"SimulationName": m["name"].split("-")[0]}
    # deep copies: editing one pod leaves the others alone
    pods[0]["spec"]["containers"][0]["resources"]["requests"]["cpu"] = 7
    assert pods[1]["spec"]["containers"][0]["resources"]["requests"]["cpu"] == 1
    u = scheduler.expand_simulation_pods(spec, uid="uuid")
    assert all(re.fullmatch(r"[0-9a-f-]{36}", p["metadata"]["name"]) for p in u)
    assert len({p["metadata"]["uid"] for p in u}) == 20


def test_pod_requirement_strings():
    """getResourceRequest + Quantity.String: the README's "CPU: 1, Memory: 1" and
    "CPU: 100, Memory: 1k" rows."""
    a, b = (scheduler.expand_simulation_pods([s])[0] for s in _podspec())
    ra, rb = report.resource_request(a), report.resource_request(b)
    assert "CPU: %s, Memory: %s" % (ra["cpu"], ra["memory"]) == "CPU: 1, Memory: 1"
    assert "CPU: %s, Memory: %s" % (rb["cpu"], rb["memory"]) == "CPU: 100, Memory: 1k"


@pytest.mark.parametrize("reqs,cpu,mem", [
    ([{}], "0", "0"),
    ([{"cpu": "100m"}, {"cpu": "200m"}], "300m", "0"),
    ([{"cpu": "1.5"}], "1500m", "0"),
    ([{"memory": "1Gi"}, {"memory": "512Mi"}], "0", "1536Mi"),
    ([{"memory": "1Gi"}, {"memory": "1G"}], "0", "2073741824"),   # last container's DecimalSI
    ([{"memory": "1G"}, {"memory": "1Gi"}], "0", "2073741824"),   # BinarySI, not a multiple of 1024
    ([{"memory": "1G"}, {"memory": "0"}], "0", "1G"),              # a zero quantity keeps the sum's format
    ([{"memory": "500"}], "0", "500"),
    ([{"memory": "1e3"}], "0", "1e3"),
    ([{"memory": "2048"}, {"memory": "0Ki"}], "0", "2048"),
    ([{"cpu": "2", "memory": "3Mi"}, {"cpu": "500m", "memory": "1Mi"}], "2500m", "4Mi"),
])
def test_summed_quantity_strings(reqs, cpu, mem):
    pod = {"spec": {"containers": [{"resources": {"requests": r}} for r in reqs]}}
    r = report.resource_request(pod)
    assert (str(r["cpu"]), str(r["memory"])) == (cpu, mem)


def test_scalar_and_gpu_requests():
    pod = {"spec": {"containers": [{"resources": {"requests": {"example.com/foo": "2", "alpha.kubernetes.io/nvidia-gpu": "1"}}},
                                   {"resources": {"requests": {"example.com/foo": "3"}}}]}}
    r = report.resource_request(pod)
    assert r["scalar"] == {"example.com/foo": 5} and str(r["nvidia_gpu"]) == "1"
    assert report.resource_request({"spec": {"containers": [{}]}})["scalar"] is None


# ----------------------------------------------------------------------------- printer
def test_failed_pods_table_matches_readme():
    b = scheduler.expand_simulation_pods([_podspec()[1]])
    st = report.simulation_status(b, [], [(None, "0/3 nodes are available: 3 Insufficient cpu.")] * 10)
    text = report.review_text(report.get_report(st))
    succ, failed = text.split("================================= Failed Pods")
    with open(os.path.join(GOLD, "readme_failed_pods.txt")) as f:
        want = f.read()
    assert "================================= Failed Pods" + failed == want
    assert succ == ("================================= Successful Pods =================================\n"
                    "+--------------+------+\n| REQUIREMENTS | HOST |\n+--------------+------+\n"
                    "+--------------+------+\n")


def test_table_layout():
    t = report.render_table(["Requirements", "Host"], [["CPU: 1, Memory: 1", "test-1474.test.com"], ["12", "x"]])
    assert t.splitlines() == ["+-------------------+--------------------+",
                              "|   REQUIREMENTS    |        HOST        |",
                              "+-------------------+--------------------+",
                              "| CPU: 1, Memory: 1 | test-1474.test.com |",
                              "|                12 | x                  |",
                              "+-------------------+--------------------+"]
    # cells over 30 columns wrap at word boundaries into extra lines
    t = report.render_table(["Requirements", "Host"], [["CPU: 1500m, Memory: 1073741824k", "h"]])
    assert t.splitlines()[3:5] == ["| CPU: 1500m, Memory: | h    |", "| 1073741824k         |      |"]


# ----------------------------------------------------------------------------- status / stop reason
@pytest.mark.parametrize("outcomes,stop", [
    ([], "fail to get next pod: No pods left\n"),
    ([("n", None)], "fail to get next pod: No pods left\n"),
    ([("n", None), (None, "x")], "Fail to get next pod: No pods left\n"),
    ([(None, "x"), ("n", None)], "fail to get next pod: No pods left\n"),
])
def test_stop_reason(outcomes, stop):
    pods = [{"metadata": {"name": "p%d" % i}, "spec": {}} for i in range(len(outcomes))]
    st = report.simulation_status(pods, [], outcomes)
    assert st.stop_reason == stop
    rv = report.get_report(st)
    assert rv["fail_reason"] == {"fail_type": "Stopped", "fail_message": stop}


def test_status_objects():
    pods = [{"metadata": {"name": "a", "uid": "u-a"}, "spec": {}}, {"metadata": {"name": "b"}, "spec": {}}]
    running = [{"metadata": {"name": "r"}, "spec": {"nodeName": "n1"}, "status": {"phase": "Running"}}]
    st = report.simulation_status(pods, running, [("n2", None), (None, "0/1 nodes are available: 1 Insufficient cpu.")])
    assert pods[0]["spec"] == {}                   # the queue's objects are not modified
    assert st.successful[0]["spec"]["nodeName"] == "n2" and st.successful[0]["status"]["phase"] == "Running"
    f = st.failed[0]["status"]
    assert f["reason"] == "Unschedulable"
    assert f["conditions"] == [{"type": "PodScheduled", "status": "False", "reason": "Unschedulable",
                                "message": "0/1 nodes are available: 1 Insufficient cpu."}]
    rv = report.get_report(st)["review"]
    assert [p["host"] for p in rv["success"]["status"]["pods"]] == ["n2"]
    assert rv["success"]["status"]["pods"][0]["pod_uid"] == "u-a"
    assert list(rv["failed"]["status"]["reason_summary"]) == ["Unschedulable"]
    assert [p["host"] for p in rv["scheduled"]["status"]["pods"]] == ["n1"]
    assert list(rv["success"]["status"]["reason_summary"]) == [""]


def test_oracle_end_to_end_report():
    """etc/pod.yaml on three 4-CPU nodes: the B pods (100 CPUs) are popped first and all fail,
    then the A pods spread over the nodes; the last pod popped (A-0) binds."""
    sim = scheduler.expand_simulation_pods(_podspec())
    rv = _oracle_report(_nodes(3), [], sim)
    text = report.review_text(rv)
    assert "\t- Unschedulable: 10\n" in text
    assert text.count("| CPU: 100, Memory: 1k |      |") == 10
    assert text.count("| CPU: 1, Memory: 1 | node-") == 10
    assert rv["fail_reason"]["fail_message"] == "fail to get next pod: No pods left\n"
    msgs = {p["status"]["conditions"][0]["message"] for p in rv["review"]["failed"]["spec"]["pods"]}
    assert msgs == {"0/3 nodes are available: 3 Insufficient cpu."}


# ----------------------------------------------------------------------------- checkpoint / CLI
def _write(tmp_path, name, obj):
    p = tmp_path / name
    p.write_text(json.dumps(obj) if not isinstance(obj, str) else obj)
    return str(p)


def test_checkpoint_loader(tmp_path):
    nodes = _nodes(2)
    pods = [{"metadata": {"name": "r"}, "spec": {"nodeName": "node-0", "containers": [{}]}}]
    n, p = scheduler.load_checkpoint(_write(tmp_path, "nodes.json", nodes), _write(tmp_path, "pods.json", pods))
    assert n == nodes and p == pods
    n, p = scheduler.load_checkpoint(_write(tmp_path, "nodes.json", nodes))
    assert p == []
    with pytest.raises(abi.KsimError):
        scheduler.load_checkpoint(_write(tmp_path, "bad.json", {"items": []}))
    with pytest.raises(ValueError):
        scheduler.load_checkpoint(_write(tmp_path, "broken.json", "[{"))


def test_cli_refuses_kubeconfig_and_bad_files(tmp_path, capsys):
    spec = os.path.join(GOLD, "etc_pod.yaml")
    nodes = _write(tmp_path, "nodes.json", _nodes(1))
    assert cli.main(["--podspec", spec, "--nodes", nodes, "--kubeconfig", "/x"]) == 1
    assert "--kubeconfig" in capsys.readouterr().err
    assert cli.main(["--podspec", spec, "--nodes", str(tmp_path / "missing.json")]) == 1
    assert "Failed to start scheduler simulator" in capsys.readouterr().err
    with pytest.raises(SystemExit):
        cli.parse_args(["--nodes", nodes])        # --podspec is required


# ----------------------------------------------------------------------------- GPU: same report
@pytest.mark.gpu
@pytest.mark.parametrize("n_nodes,running", [(3, 0), (1, 0), (7, 5)])
def test_gpu_report_matches_oracle(n_nodes, running):
    nodes = _nodes(n_nodes)
    run = [{"metadata": {"name": "r%d" % i, "uid": "r%d" % i}, "spec": {"nodeName": "node-%d" % (i % n_nodes),
            "containers": [{"resources": {"requests": {"cpu": "1", "memory": "1Gi"}}}]}, "status": {"phase": "Running"}}
           for i in range(running)]
    sim = scheduler.expand_simulation_pods(_podspec())
    want = _oracle_report(nodes, run, sim)
    rep = scheduler.ClusterCapacity(nodes, run, sim, provider_name=PROVIDER).run()
    assert report.review_text(rep.review) == report.review_text(want)
    assert rep.stop_reason == want["fail_reason"]["fail_message"]
    for k in ("failed", "success", "scheduled"):
        got = [(p["pod_name"], p["host"], p["reason"]) for p in rep.review["review"][k]["status"]["pods"]]
        exp = [(p["pod_name"], p["host"], p["reason"]) for p in want["review"][k]["status"]["pods"]]
        assert got == exp, k
    gm = [p["status"]["conditions"][0]["message"] for p in rep.review["review"]["failed"]["spec"]["pods"]]
    em = [p["status"]["conditions"][0]["message"] for p in want["review"]["failed"]["spec"]["pods"]]
    assert gm == em


@pytest.mark.gpu
def test_gpu_cli_end_to_end(tmp_path):
    nodes = _nodes(3)
    spec = os.path.join(GOLD, "etc_pod.yaml")
    nf = _write(tmp_path, "nodes.json", nodes)
    buf = io.StringIO()
    with redirect_stdout(buf):
        assert cli.main(["--podspec", spec, "--nodes", nf]) == 0
    want = report.review_text(_oracle_report(nodes, [], scheduler.expand_simulation_pods(_podspec())))
    assert buf.getvalue() == want
    buf = io.StringIO()
    with redirect_stdout(buf):
        assert cli.main(["--podspec", spec, "--nodes", nf, "--json"]) == 0
    rv = json.loads(buf.getvalue())
    assert rv["fail_reason"]["fail_message"] == "fail to get next pod: No pods left\n"
    assert len(rv["review"]["success"]["status"]["pods"]) == 10
