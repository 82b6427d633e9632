#!/usr/bin/env python3
"""Median per dispatch of every rocprofv3 --pmc counter, per kernel name (template arguments
kept), over all pass directories under a root: pmc_by_kernel.py <root> [filter-substring ...]."""
import csv
import glob
import json
import os
import statistics
import sys


def main():
    root = sys.argv[1]
    keep = sys.argv[2:]
    per = {}
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                if keep and not any(k in name for k in keep):
                    continue
                did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                d = per.setdefault(name, {}).setdefault(r["Counter_Name"], {})
                d[did] = d.get(did, 0.0) + float(r["Counter_Value"])
    out = {k: {c: statistics.median(v.values()) for c, v in cs.items()} | {"dispatches": max(len(v) for v in cs.values())}
           for k, cs in per.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
