"""Summarise rocprofv3 --pmc counter CSVs under a gpurun_out/<tag> directory: per kernel, the
per-dispatch average of every counter collected (FETCH_SIZE / WRITE_SIZE are in KB)."""
import csv
import glob
import json
import os
import sys


def summarise(root):
    out = {}
    for f in glob.glob(os.path.join(root, "*", "*counter_collection.csv")):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0]
            d = out.setdefault(k, {})
            d.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
    return {k: {c: {"dispatches": len(v), "avg": sum(v) / len(v)} for c, v in d.items()} for k, d in out.items()}


if __name__ == "__main__":
    s = summarise(sys.argv[1])
    print(json.dumps(s, indent=1))
    json.dump(s, open(os.path.join(sys.argv[1], "pmc_summary.json"), "w"), indent=1)
