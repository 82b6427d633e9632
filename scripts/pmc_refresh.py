#!/usr/bin/env python3
"""Summarise scripts/pmc_refresh.sh's passes into profiles/pmc_traffic.json (and copies for profiles/<round>/pmc/).

  python3 scripts/pmc_refresh.py gpurun_out/<tag> [--profiles profiles/r05/pmc] [--out profiles/pmc_traffic.json]

Each pass ran scripts/pmc_workloads.py, whose plan.json lists every pollnet kernel call in order (label, kernel
families).  The pass's dispatches of those families, in Dispatch_Id order, are matched one to one to that list
(the script stops if the count or a family differs); each label's calls then give per-call medians of every
counter.  Bytes per call, as the MI355X guide's HBM section prescribes:
  read  = FETCH_SIZE (KiB) x 1024 x factor, factor = the calibration stream read's known bytes / its FETCH_SIZE
          (gfx950 FETCH_SIZE under-reports wide streaming reads);
  write = WRITE_SIZE (KiB) x 1024;
  EA    = 32/64/128 x TCC_EA0_RDREQ_{32B,64B,128B} + 64 x WRREQ_64B + 32 x (WRREQ - WRREQ_64B).
Every entry records the code hash of each kernel its counters summed over (pollnet_amd/codehash.py), taken from the
library in this tree; the plan's lib_sha256 must equal this tree's library, so the hashes are of the code that ran."""
import argparse
import collections
import csv
import glob
import hashlib
import json
import os
import shutil
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
TUNING = os.path.join(ROOT, "pollnet_amd", "libpollnet_amd_tuning.so")
FAMILIES = ("rx_classify_kernel", "match_streams_mask_kernel", "tx_fill_kernel", "tx_patch_kernel",
            "calib_stream_read_kernel", "tx_patch_wt_kernel", "tx_l2_release_kernel", "tx_patch_sector_kernel")


def family(name):
    for f in FAMILIES:
        if f + "<" in name or f + "(" in name:
            return f
    return None


def dispatches(pass_dir, kind):
    """[(dispatch_id, kernel name, {counter: value} or (start, end))] of the pollnet families, in order."""
    per = collections.OrderedDict()
    if kind == "pmc":
        files = glob.glob(os.path.join(pass_dir, "**", "*counter_collection.csv"), recursive=True)
        for f in files:
            for r in csv.DictReader(open(f)):
                if family(r["Kernel_Name"]) is None:
                    continue
                did = int(r["Dispatch_Id"])
                d = per.setdefault(did, [r["Kernel_Name"], collections.defaultdict(float)])
                d[1][r["Counter_Name"]] += float(r["Counter_Value"])
    else:
        files = glob.glob(os.path.join(pass_dir, "**", "*kernel_trace.csv"), recursive=True)
        for f in files:
            for r in csv.DictReader(open(f)):
                if family(r["Kernel_Name"]) is None:
                    continue
                per[int(r["Dispatch_Id"])] = [r["Kernel_Name"], (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))]
    assert files, f"no rocprofv3 CSV under {pass_dir}"
    return [(k, v[0], v[1]) for k, v in sorted(per.items())]


def label_calls(root, name, kind):
    """{label: [[(kernel name, data) per kernel of the call] per call]} for one pass."""
    plan = json.load(open(os.path.join(root, name, "plan.json")))
    ds = dispatches(os.path.join(root, name), kind)
    want = [(lab, fam) for lab, fams in plan["calls"] for fam in fams]
    assert len(ds) == len(want), f"{name}: {len(ds)} pollnet dispatches, the plan lists {len(want)}"
    out = collections.defaultdict(list)
    i = 0
    for lab, fams in plan["calls"]:
        call = []
        for fam in fams:
            did, kname, data = ds[i]
            assert family(kname) == fam, f"{name}: dispatch {did} is {kname}, the plan expects {fam}"
            call.append((kname, data))
            i += 1
        out[lab].append(call)
    return plan, out


def med_counter(calls, counter, kernel_fam=None):
    vals = []
    for call in calls:
        s = 0.0
        for kname, data in call:
            if kernel_fam is None or family(kname) == kernel_fam:
                s += data.get(counter, 0.0)
        vals.append(s)
    return statistics.median(vals)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("root")
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--profiles", default=None, help="copy the per-pass summaries and the trace stats here")
    args = ap.parse_args()
    from pollnet_amd import codehash

    passes = {p: label_calls(args.root, p, "pmc") for p in ("fetch", "write", "ea", "eaw")}
    plan = passes["fetch"][0]
    with open(os.path.join(ROOT, "pollnet_amd", "libpollnet_amd.so"), "rb") as f:
        here = hashlib.sha256(f.read()).hexdigest()
    for p, (pl, _) in passes.items():
        assert pl["lib_sha256"] == here, f"pass {p} ran another build of libpollnet_amd.so than this tree's"
        assert all(pl["gates"].values()), f"pass {p}: a correctness gate failed: {pl['gates']}"
    fetch, write, ea, eaw = (passes[p][1] for p in ("fetch", "write", "ea", "eaw"))
    factor = plan["workloads"]["calib"]["bytes_per_launch"] / (med_counter(fetch["calib"], "FETCH_SIZE") * 1024)
    trace = None
    if os.path.isdir(os.path.join(args.root, "trace")):
        _, trace = label_calls(args.root, "trace", "trace")

    def entry(label, fam=None):
        w = plan["workloads"][label]
        n = w.get("frames", plan["frames"])
        read = med_counter(fetch[label], "FETCH_SIZE", fam) * 1024 * factor
        wr = med_counter(write[label], "WRITE_SIZE", fam) * 1024
        cnt = {c: med_counter(ea[label], c, fam) for c in ("TCC_EA0_RDREQ_sum", "TCC_EA0_RDREQ_32B_sum",
                                                             "TCC_EA0_RDREQ_64B_sum", "TCC_EA0_RDREQ_128B_sum")}
        cnt.update({c: med_counter(eaw[label], c, fam) for c in ("TCC_EA0_WRREQ_sum", "TCC_EA0_WRREQ_64B_sum",
                                                                   "TCC_EA0_RDREQ_DRAM_sum")})
        rd = 32 * cnt["TCC_EA0_RDREQ_32B_sum"] + 64 * cnt["TCC_EA0_RDREQ_64B_sum"] + 128 * cnt["TCC_EA0_RDREQ_128B_sum"]
        w64 = cnt["TCC_EA0_WRREQ_64B_sum"]
        ea_w = 64 * w64 + 32 * (cnt["TCC_EA0_WRREQ_sum"] - w64)
        names = {k for call in fetch[label] for k, _ in call if fam is None or family(k) == fam}
        e = {"workload": w["workload"], "frames_per_launch": n,
             "hbm_read_bytes_per_launch": int(read), "hbm_write_bytes_per_launch": int(wr),
             "hbm_bytes_per_launch": int(read + wr),
             "fetch_correction_factor": round(factor, 4),
             "ea_request_counters": {k: round(v, 1) for k, v in cnt.items()},
             "ea_bytes_per_launch": int(rd + ea_w),
             "ea_read_requests_per_frame": round(cnt["TCC_EA0_RDREQ_sum"] / n, 4),
             "ea_read_128B_per_frame": round(cnt["TCC_EA0_RDREQ_128B_sum"] / n, 4),
             "ea_write_requests_per_frame": round(cnt["TCC_EA0_WRREQ_sum"] / n, 4),
             "ea_write_64B_per_frame": round(w64 / n, 4),
             "calls_measured": len(fetch[label]),
             "kernels": codehash.matching(names, TUNING if label.startswith("x_") else None)}
        if fam is None:
            algo = w["algorithmic_bytes_per_launch"]
            e["algorithmic_bytes_per_launch"] = algo
            e["traffic_over_algorithmic"] = round((read + wr) / algo, 4)
        if trace is not None and label in trace:
            durs = []
            for call in trace[label]:
                durs.append(sum(t1 - t0 for k, (t0, t1) in call if fam is None or family(k) == fam) / 1e3)
            e["trace_kernel_us_median"] = round(statistics.median(durs), 2)
        e["source"] = os.path.relpath(args.profiles, ROOT) if args.profiles else args.root
        e["method"] = ("scripts/pmc_refresh.sh: scripts/pmc_workloads.py under rocprofv3, --pmc FETCH_SIZE / WRITE_SIZE / "
                       "EA read requests / EA write requests in separate passes, per-call medians over the label's calls, "
                       "FETCH scaled by the same pass's calibration stream read; scripts/pmc_refresh.py")
        return e

    d = {}
    if os.path.exists(args.out):
        d = json.load(open(args.out))
    new, exper = {}, {}
    for label in plan["workloads"]:
        if label == "calib":
            continue
        if label.startswith(("x_", "uncached_")):  # experiments: their own file, never pmc_traffic.json
            key, sub = label.split("/") if "/" in label else (label, "all")
            t = entry(label)
            t["per_kernel"] = {fam: entry(label, fam) for fam in sorted({family(k) for c in fetch[label] for k, _ in c})}
            for v in t["per_kernel"].values():
                v.pop("source", None)
                v.pop("method", None)
            exper.setdefault(key, {})[sub] = t
            continue
        if label.startswith("tx_"):
            key, sub = label.split("/")
            t = entry(label)
            t["per_kernel"] = {fam: entry(label, fam) for fam in ("tx_fill_kernel", "tx_patch_kernel")}
            for v in t["per_kernel"].values():
                v.pop("source", None)
                v.pop("method", None)
            new.setdefault(key, {})[sub] = t
        else:
            new[label] = entry(label)
    for k, v in new.items():
        if isinstance(d.get(k), dict) and k.startswith("tx_"):
            d[k].update(v)
        else:
            d[k] = v
    with open(args.out, "w") as f:
        json.dump(d, f, indent=1)
    if args.profiles:
        os.makedirs(args.profiles, exist_ok=True)
        with open(os.path.join(args.profiles, "pmc_entries.json"), "w") as f:
            json.dump(new, f, indent=1)
        if exper:
            with open(os.path.join(args.profiles, "experiments.json"), "w") as f:
                json.dump(exper, f, indent=1)
        with open(os.path.join(args.profiles, "gates.json"), "w") as f:
            json.dump({"lib_sha256": plan["lib_sha256"], "gates": plan["gates"]}, f, indent=1)
        for st in glob.glob(os.path.join(args.root, "trace", "**", "*kernel_stats.csv"), recursive=True):
            shutil.copy(st, os.path.join(args.profiles, "trace_kernel_stats.csv"))
    summary = {k: ({s: (e["hbm_bytes_per_launch"], e["traffic_over_algorithmic"]) for s, e in v.items()}
                   if k.startswith("tx_") else (v["hbm_bytes_per_launch"], v["traffic_over_algorithmic"]))
               for k, v in new.items()}
    print(json.dumps(summary, indent=1))
    if exper:
        print(json.dumps({k: {s: (e["hbm_bytes_per_launch"], e["ea_write_requests_per_frame"], e["ea_write_64B_per_frame"],
                                  e.get("trace_kernel_us_median")) for s, e in v.items()} for k, v in exper.items()}, indent=1))


if __name__ == "__main__":
    main()
