#!/usr/bin/env python3
"""Per-wave medians of the SQ counters of scripts/sq_probe_pmc.sh, per RX kernel variant (ABL template value):
sq_summarize.py <pass_root> [configs...] > summary.json"""
import csv
import glob
import json
import re
import statistics
import sys


def main():
    root = sys.argv[1]
    cfgs = [int(c) for c in sys.argv[2:]] or [3, 5]
    out = {}
    for c in cfgs:
        per = {}
        for f in glob.glob(f"{root}/c{c}_p*/**/*counter_collection.csv", recursive=True):
            with open(f) as fh:
                for r in csv.DictReader(fh):
                    m = re.search(r"rx_classify_kernel<0, 1, (\d+),", r.get("Kernel_Name", ""))
                    if not m:
                        continue
                    d = per.setdefault(m.group(1), {}).setdefault(r["Counter_Name"], {})
                    d[r["Dispatch_Id"]] = d.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
        out[f"c{c}"] = {}
        for abl, cs in per.items():
            w = statistics.median(cs["SQ_WAVES"].values()) if "SQ_WAVES" in cs else 1.0
            out[f"c{c}"][abl] = {k: round(statistics.median(v.values()) / w, 1) for k, v in cs.items()}
    json.dump(out, sys.stdout, indent=1)


if __name__ == "__main__":
    main()
