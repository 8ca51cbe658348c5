"""Summarise rocprofv3 --pmc counter CSVs under a gpurun_out/<tag> directory: per kernel, the
per-dispatch average of every counter collected (FETCH_SIZE / WRITE_SIZE are in KB).

  python tools/pmc_summary.py <dir>                       # per-kernel summary → <dir>/pmc_summary.json
  python tools/pmc_summary.py <dir> --record <workload> <kernel substring> <node-evals per dispatch> <profiled command>
      → also writes the bench.py record (profiles/r3/pmc_<workload>.json format) for that kernel:
        HBM bytes per node-eval = (FETCH_SIZE x 2 + WRITE_SIZE) x 1024 / node-evals, FETCH_SIZE
        doubled as MI355X_MICROARCH.md prescribes for gfx950 (it reports half of wide streamed reads)."""
import csv
import glob
import json
import os
import sys


def kernel_name(full):
    """Strip the trailing parameter list: 'void k<1, false>(A, B)' → 'void k<1, false>'."""
    s = full.strip()
    if not s.endswith(")"):
        return s
    depth = 0
    for i in range(len(s) - 1, -1, -1):
        if s[i] == ")":
            depth += 1
        elif s[i] == "(":
            depth -= 1
            if depth == 0:
                return s[:i]
    return s


def summarise(root):
    out = {}
    for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = kernel_name(r["Kernel_Name"])
            d = out.setdefault(k, {})
            d.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: {c: {"dispatches": len(v), "avg": sum(v) / len(v)} for c, v in d.items()} for k, d in out.items()}


if __name__ == "__main__":
    s = summarise(sys.argv[1])
    json.dump(s, open(os.path.join(sys.argv[1], "pmc_summary.json"), "w"), indent=1)
    if len(sys.argv) > 2 and sys.argv[2] == "--record":
        workload, sub, evals, cmd = sys.argv[3], sys.argv[4], float(sys.argv[5]), sys.argv[6]
        ks = [k for k in s if sub in k]
        assert len(ks) == 1, ks
        d = s[ks[0]]
        fetch, write = d["FETCH_SIZE"]["avg"], d["WRITE_SIZE"]["avg"]
        rec = {"workload": workload, "kernel": ks[0], "profiled": cmd, "node_evals_per_dispatch": evals,
               "dispatches": d["FETCH_SIZE"]["dispatches"], "fetch_size_kb": fetch, "write_size_kb": write,
               "correction": "FETCH_SIZE x2 (gfx950 reports half of wide streamed reads), KB = 1024 B",
               "hbm_bytes_per_node_eval": (2 * fetch + write) * 1024 / evals,
               "fetch_bytes_per_node_eval": 2 * fetch * 1024 / evals}
        print(json.dumps(rec, indent=1))
    else:
        print(json.dumps(s, indent=1))
