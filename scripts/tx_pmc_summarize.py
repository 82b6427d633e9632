#!/usr/bin/env python3
"""HBM bytes per pn_tx_fill call from scripts/gpu_tx_pmc.sh passes (one dir per frame_off):
FETCH_SIZE (KiB, x the same run's calibration factor) + WRITE_SIZE (KiB) of tx_fill_kernel and
tx_patch_kernel, cross-checked with the EA request counts; merged into profiles/pmc_traffic.json
under "tx_c2_n1048576".
  tx_pmc_summarize.py <dir_off2> <dir_off14> [profiles/pmc_traffic.json]"""
import csv
import glob
import json
import os
import statistics
import sys

N, ALGO = 1 << 20, 1504 << 20


def per_kernel(root):
    res = {}
    for d in ("fetch", "write", "ea", "eaw"):
        per = {}
        for f in glob.glob(os.path.join(root, d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                k = r["Kernel_Name"]
                kind = ("calib" if "calib_stream_read" in k else "fill" if "tx_fill_kernel" in k else
                        "patch" if "tx_patch_kernel<0, 0>" in k or "tx_patch_kernel<0>" in k else None)
                if kind is None:
                    continue
                did = r.get("Dispatch_Id") or r.get("Correlation_Id")
                per.setdefault((kind, r["Counter_Name"]), {}).setdefault(did, 0.0)
                per[(kind, r["Counter_Name"])][did] += float(r["Counter_Value"])
        for (k, c), v in per.items():
            res.setdefault(k, {})[c] = statistics.median(v.values())
    return res


def summarize(root, off):
    k = per_kernel(root)
    calib_bytes = 2048 * N
    factor = calib_bytes / (k["calib"]["FETCH_SIZE"] * 1024)
    rd = sum(k[x]["FETCH_SIZE"] * 1024 * factor for x in ("fill", "patch"))
    wr = sum(k[x]["WRITE_SIZE"] * 1024 for x in ("fill", "patch"))
    ea_rd = sum(k[x].get("TCC_EA0_RDREQ_128B_sum", 0) * 128 + k[x].get("TCC_EA0_RDREQ_64B_sum", 0) * 64
                for x in ("fill", "patch"))
    ea_wr = sum(k[x].get("TCC_EA0_WRREQ_64B_sum", 0) * 64 +
                (k[x].get("TCC_EA0_WRREQ_sum", 0) - k[x].get("TCC_EA0_WRREQ_64B_sum", 0)) * 32 for x in ("fill", "patch"))
    return {
        "workload": "C2 frames (tot_len 1500), both checksums scrambled; pn_tx_fill PN_TX_TCP",
        "frame_off": off, "frames_per_launch": N,
        "fetch_correction_factor": round(factor, 4),
        "per_kernel": {x: {c: v for c, v in k[x].items()} for x in ("fill", "patch")},
        "hbm_read_bytes_per_launch": int(rd), "hbm_write_bytes_per_launch": int(wr),
        "hbm_bytes_per_launch": int(rd + wr), "algorithmic_bytes_per_launch": ALGO,
        "traffic_over_algorithmic": round((rd + wr) / ALGO, 4),
        "ea_bytes_per_launch": int(ea_rd + ea_wr),
        "write_requests_per_frame": round(sum(k[x].get("TCC_EA0_WRREQ_sum", 0) for x in ("fill", "patch")) / N, 4),
        "method": "scripts/tx_pmc_probe.py under rocprofv3: --pmc FETCH_SIZE / WRITE_SIZE / EA read / EA write in "
                  "separate passes; FETCH scaled by the same run's calibration stream read of a known byte count",
    }


def main():
    out = sys.argv[3] if len(sys.argv) > 3 else "profiles/pmc_traffic.json"
    d = json.load(open(out))
    d["tx_c2_n1048576"] = {"frame_off_2": summarize(sys.argv[1], 2), "frame_off_14": summarize(sys.argv[2], 14)}
    json.dump(d, open(out, "w"), indent=1)
    print(json.dumps({k: (v["hbm_bytes_per_launch"], v["traffic_over_algorithmic"], v["write_requests_per_frame"])
                      for k, v in d["tx_c2_n1048576"].items()}))


if __name__ == "__main__":
    main()
