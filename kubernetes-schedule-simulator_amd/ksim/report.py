"""The simulator's report (pkg/framework/report.go:96-245) and its text printer.

Status — framework.Status (report.go:240-245): successful pods in bind order (spec.nodeName set,
phase Running, simulator.go:108-145), failed pods (phase Pending, a PodScheduled=False condition
with reason Unschedulable and the FitError text as its message, status.reason = "Unschedulable",
simulator.go:163-185), the already-running pods of the snapshot (AddScheduledPods, :96,321) and
the stop reason written when the queue runs dry (simulator.go:137, :169, :205).

get_report — GetReport (report.go:168-174): per review ("failed", "success", "scheduled") the pods'
requirements (getResourceRequest, :96-129: cpu / memory / nvidia-gpu summed over containers as
Quantities, scalar resources as int64) and status (PodReviewResult per pod and the ReasonSummary
keyed by status.reason); FailReason {Stopped, StopReason}.

cluster_capacity_review_print — ClusterCapacityReviewPrint (report.go:201-237) with tablewriter's
default table layout.
"""
from __future__ import annotations

import io
import re
import sys
from dataclasses import dataclass, field
from fractions import Fraction

from . import quantity
from .ingest import GPU, is_scalar_resource

CPU, MEM = "cpu", "memory"


@dataclass
class Status:
    successful: list = field(default_factory=list)
    failed: list = field(default_factory=list)
    scheduled: list = field(default_factory=list)
    stop_reason: str = ""


NO_PODS_LEFT = "No pods left"                      # store.go:229
ERR_NO_NODES = "no nodes available to schedule pods"  # generic_scheduler.go:64


def simulation_status(order, running, outcomes) -> Status:
    """The Status a ClusterCapacity run leaves: `order` the simulation pods in pop order,
    `running` the snapshot's pods, `outcomes` per popped pod (node name, None) when bound or
    (None, error text) when scheduling failed.
    - Bind (simulator.go:108-145): a copy with spec.nodeName and phase Running → successful.
    - Update (simulator.go:163-185): a copy with the PodScheduled=False condition (reason
      Unschedulable, message = the error), status.reason Unschedulable → failed.
    - the queue runs dry inside the next Bind / Update: "fail to get next pod: ..." after a
      bind or on an empty queue, "Fail to get next pod: ..." after a failure (:137, :169, :205)."""
    import copy
    st = Status(scheduled=list(running))
    for pod, (node, msg) in zip(order, outcomes):
        pod = copy.deepcopy(pod)
        if node is not None:
            pod.setdefault("spec", {})["nodeName"] = node
            pod.setdefault("status", {})["phase"] = "Running"
            st.successful.append(pod)
        else:
            ps = pod.setdefault("status", {})
            ps.setdefault("conditions", []).append({"type": "PodScheduled", "status": "False",
                                                   "reason": "Unschedulable", "message": msg})
            ps["reason"] = "Unschedulable"
            st.failed.append(pod)
    last_failed = len(outcomes) > 0 and outcomes[-1][0] is None
    st.stop_reason = "%sail to get next pod: %s\n" % ("F" if last_failed else "f", NO_PODS_LEFT)
    return st


class Q:
    """A summed Quantity: exact value + the Format Quantity.Add keeps (report.go:107-117: the
    container's quantity is added to the running sum, so the last non-zero container's format
    wins; a zero quantity takes the other operand's)."""

    def __init__(self, value=Fraction(0), form=quantity.DECIMAL_SI):
        self.value, self.form = Fraction(value), form

    def add_container(self, q):
        v = quantity.parse(q)
        form = quantity.fmt(q)
        if v == 0:
            form = self.form
        self.value, self.form = self.value + v, form

    def __str__(self):
        return quantity.canonical(self.value, self.form)

    def is_zero(self):
        return self.value == 0


def resource_request(pod):
    """getResourceRequest (report.go:96-129)."""
    cpu = Q(0, quantity.DECIMAL_SI)
    mem = Q(0, quantity.BINARY_SI)
    gpu = Q(0, quantity.DECIMAL_SI)
    scalar = None
    for c in (pod.get("spec") or {}).get("containers") or []:
        for name, q in ((c.get("resources") or {}).get("requests") or {}).items():
            if name == MEM:
                mem.add_container(q)
            elif name == CPU:
                cpu.add_container(q)
            elif name == GPU:
                gpu.add_container(q)
            elif is_scalar_resource(name):
                scalar = scalar or {}
                scalar[name] = scalar.get(name, 0) + quantity.value(q)
    return {"cpu": cpu, "memory": mem, "nvidia_gpu": gpu, "scalar": scalar}


def _review(pods):
    reqs = [{"pod_name": (p.get("metadata") or {}).get("name", ""), "resources": resource_request(p),
             "node_selector": (p.get("spec") or {}).get("nodeSelector")} for p in pods]
    summary, results = {}, []
    for p, r in zip(pods, reqs):
        prr = {"pod_uid": (p.get("metadata") or {}).get("uid", ""), "pod_name": r["pod_name"],
               "host": (p.get("spec") or {}).get("nodeName", ""), "reason": (p.get("status") or {}).get("reason", ""),
               "resources": r["resources"]}
        summary.setdefault(prr["reason"], []).append(prr)
        results.append(prr)
    return {"spec": {"pods": pods, "pod_requirements": reqs},
            "status": {"pods": results, "reason_summary": summary}}


def get_report(status: Status):
    """GetReport (report.go:168-174)."""
    return {"review": {"failed": _review(status.failed), "success": _review(status.successful),
                       "scheduled": _review(status.scheduled)},
            "fail_reason": {"fail_type": "Stopped", "fail_message": status.stop_reason}}


# tablewriter (github.com/olekukonko/tablewriter, a Gopkg dependency whose source is not vendored in
# the reference): NewWriter defaults are auto-wrap at 30 display columns (minimum-raggedness word
# wrap), header titles upper-cased and centred, cells matching ^-*\d*\.?\d*$ right-aligned, others
# left-aligned, one space of padding, '+' / '-' / '|' borders.  The layout is pinned only by the
# reference README's sample output (header centring, border widths); wrapping is parity-unpinned.
MAX_ROW_WIDTH = 30
_PENALTY = 100000
_DECIMAL = re.compile(r"^-*\d*\.?\d*$")


def wrap_words(words, spc, lim, pen=_PENALTY):
    """Minimum-raggedness word wrap: line cost (lim - len)^2, `pen` added to over-long lines,
    the last line free."""
    n = len(words)
    length = [[0] * n for _ in range(n)]
    for i in range(n):
        length[i][i] = len(words[i])
        for j in range(i + 1, n):
            length[i][j] = length[i][j - 1] + spc + len(words[j])
    nbrk, cost = [0] * n, [2**31 - 1] * n
    for i in range(n - 1, -1, -1):
        if length[i][n - 1] <= lim:
            cost[i], nbrk[i] = 0, n
            continue
        for j in range(i + 1, n):
            d = lim - length[i][j - 1]
            c = d * d + cost[j] + (pen if length[i][j - 1] > lim else 0)
            if c < cost[i]:
                cost[i], nbrk[i] = c, j
    lines, i = [], 0
    while i < n:
        lines.append(words[i:nbrk[i]])
        i = nbrk[i]
    return lines


def wrap_string(s, lim=MAX_ROW_WIDTH):
    words = s.replace("\n", " ").split(" ")
    lim = max([lim] + [len(w) for w in words])
    return [" ".join(l) for l in wrap_words(words, 1, lim)] or [""]


def render_table(header, rows):
    hdr = [h.replace("_", " ").replace(".", " ").strip().upper() for h in header]
    width = [len(h) for h in hdr]
    cells = []
    for r in rows:
        lines = [wrap_string(c) for c in r]
        for i, ls in enumerate(lines):
            width[i] = max([width[i]] + [len(x) for x in ls])
        cells.append(lines)
    sep = "+" + "+".join("-" * (w + 2) for w in width) + "+"

    def center(s, w):
        left = (w - len(s)) // 2
        return " " * left + s + " " * (w - len(s) - left)

    def cell(s, w):
        return s.rjust(w) if _DECIMAL.match(s.strip()) else s.ljust(w)

    out = [sep, "| " + " | ".join(center(h, w) for h, w in zip(hdr, width)) + " |", sep]
    for lines in cells:
        for k in range(max(len(ls) for ls in lines)):
            out.append("| " + " | ".join(cell(ls[k] if k < len(ls) else "", w) for ls, w in zip(lines, width)) + " |")
    out.append(sep)
    return "\n".join(out) + "\n"


def _header(title):
    return "================================= %s =================================\n" % title


def _distribute(review):
    rows = [["CPU: %s, Memory: %s" % (s["resources"]["cpu"], s["resources"]["memory"]), s["host"]]
            for s in review["status"]["pods"]]
    return render_table(["Requirements", "Host"], rows)


def cluster_capacity_review_print(report, out=None):
    """ClusterCapacityReviewPrint (report.go:234-237): successful pods, then failed pods with the
    reason summary."""
    out = out or sys.stdout
    out.write(_header("Successful Pods"))
    out.write(_distribute(report["review"]["success"]))
    failed = report["review"]["failed"]
    out.write(_header("Failed Pods"))
    out.write("Pods summary:\n")
    for k, v in failed["status"]["reason_summary"].items():
        out.write("\t- %s: %d\n" % (k, len(v)))
    out.write(_distribute(failed))


def review_text(report) -> str:
    buf = io.StringIO()
    cluster_capacity_review_print(report, buf)
    return buf.getvalue()
