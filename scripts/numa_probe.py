#!/usr/bin/env python3
"""Does the host core / NUMA node the poller runs on change the zero-copy classify of a pinned ring
(the drop-in server's per-poll leg)?  The parent reads the GPU's NUMA node from sysfs and
starts one child per CPU placement (GPU-local node, a remote node, the default affinity); each child
pins itself BEFORE touching the GPU, allocates the pinned ring and records (hipHostMalloc through
torch), and times pn_classify_notify / pn_classify + sync round trips of 512 / 4096 / 16384 C4 frames
read in place.  A measurement, not part of any product path.   numa_probe.py [out.json]"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def cpulist(text):
    out = []
    for part in text.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out += list(range(int(a), int(b) + 1))
        elif part:
            out.append(int(part))
    return out


def gpu_numa():
    """(numa node, pci bdf) of the first GPU via sysfs (drm render nodes' device links)."""
    import glob

    for card in sorted(glob.glob("/sys/class/drm/card*/device")):
        try:
            vendor = open(os.path.join(card, "vendor")).read().strip()
        except OSError:
            continue
        if vendor != "0x1002":
            continue
        bdf = os.path.basename(os.path.realpath(card))
        try:
            node = int(open(os.path.join(card, "numa_node")).read().strip())
        except (OSError, ValueError):
            node = -1
        return node, bdf
    return -1, None


def child(cpus):
    os.sched_setaffinity(0, cpus)
    sys.path.insert(0, ROOT)
    import statistics
    import time

    import numpy as np
    import torch

    import pollnet_amd as pa

    p = pa.rx.GenParams.for_config(4)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    out = {"cpu": os.sched_getaffinity(0).__len__()}
    st = torch.cuda.Stream()
    word = torch.zeros(16, dtype=torch.int32, pin_memory=True)
    wnp = word.numpy()
    tok = 0
    for n in (512, 4096, 16384):
        s = pa.gen_frames(p, n)
        ring = torch.empty(n * 2048, dtype=torch.uint8, pin_memory=True)
        ring.numpy()[:] = s.reshape(-1)
        rec = torch.empty(n * 16, dtype=torch.uint8, pin_memory=True)
        ts = []
        for i in range(220):
            t0 = time.perf_counter()
            if n <= pa.rx.PN_NOTIFY_MAX_FRAMES:
                tok += 1
                ctx.classify_notify(ring, 2048, 2, n, rec, word, tok, st)
                while int(wnp[0]) != tok:
                    pass
            else:
                ctx.classify(ring, 2048, 2, n, rec, st)
                st.synchronize()
            if i >= 20:
                ts.append(time.perf_counter() - t0)
        out[str(n)] = {"us_median": round(statistics.median(ts) * 1e6, 2),
                       "pcie_gbs": round(n * 1536 / statistics.median(ts) / 1e9, 1)}
    st.synchronize()
    ctx.close()
    print(json.dumps(out))


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "--child":
        child(cpulist(sys.argv[2]))
        return
    node, bdf = gpu_numa()
    nodes = sorted(int(d[4:]) for d in os.listdir("/sys/devices/system/node") if d.startswith("node") and d[4:].isdigit())
    allowed = set(os.sched_getaffinity(0))
    res = {"gpu_bdf": bdf, "gpu_numa_node": node, "nodes": nodes, "default_affinity_cpus": len(allowed)}
    plans = {}
    for nd in nodes:
        cpus = [c for c in cpulist(open(f"/sys/devices/system/node/node{nd}/cpulist").read()) if c in allowed]
        if cpus:
            plans[f"node{nd}" + ("_gpu_local" if nd == node else "")] = cpus[:8]
    plans["default"] = sorted(allowed)
    for name, cpus in plans.items():
        r = subprocess.run([sys.executable, __file__, "--child", ",".join(map(str, cpus))], capture_output=True, text=True,
                           timeout=120)
        try:
            res[name] = json.loads(r.stdout.strip().splitlines()[-1])
        except Exception:
            res[name] = {"error": r.stderr[-400:]}
    print(json.dumps(res, indent=1))
    if len(sys.argv) > 1:
        with open(sys.argv[1], "w") as f:
            json.dump(res, f, indent=1)


if __name__ == "__main__":
    main()
