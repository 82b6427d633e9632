#!/usr/bin/env python3
"""C2 kernel time and counters by where the batch sits in HBM.

K hipMalloc'd 2-GiB buffers get the same C2 frames; each is timed in interleaved rounds (HIP
events), then classified 10 times in buffer order.  Run under `rocprofv3 --pmc ...` (one pass
per counter set, scripts/placement_pmc.sh): the last K*10 rx_classify dispatches of the pass
are that counter phase, mapped back to buffers by postprocessing (--summarize).  A
measurement, not part of any product path.

  placement_pmc.py run <out.json> [K]
  placement_pmc.py summarize <root_dir_with_pass_dirs_and_run_jsons> > summary.json
  placement_pmc.py orders <out.json> [K]   (no profiler) per buffer: the product kernel (XCD-contiguous
      group order), the same kernel in blockIdx order (tuning variant 36) and a plain stream read of
      the buffer, interleaved rounds -- is a slow placement slow for every access order, and for a
      front-to-back read of all its bytes?"""
import csv
import ctypes as C
import glob
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
REPS = 10


def run(out_path, k):
    import torch

    import pollnet_amd as pa

    n, stride, off = 1 << 20, 2048, 2
    p = pa.rx.GenParams.for_config(2)
    s = pa.gen_frames(p, n, stride, off)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    src = torch.from_numpy(s.reshape(-1)).cuda()
    hip = C.CDLL("libamdhip64.so.7")
    ptrs = []
    for _ in range(k):
        ptr = C.c_void_p()
        assert hip.hipMalloc(C.byref(ptr), C.c_size_t(n * stride)) == 0
        assert hip.hipMemcpy(ptr, C.c_void_p(src.data_ptr()), C.c_size_t(n * stride), 3) == 0
        ptrs.append(ptr.value)
    torch.cuda.synchronize()
    ref = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    res = torch.empty_like(ref)
    st = torch.cuda.current_stream()
    ctx.classify(src, stride, off, n, ref, st)
    for q in ptrs:
        ctx.classify(q, stride, off, n, res, st)
        torch.cuda.synchronize()
        assert torch.equal(res, ref)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = [[] for _ in ptrs]
    for _ in range(5):
        for i, q in enumerate(ptrs):
            ev[0].record(st)
            for _ in range(20):
                ctx.classify(q, stride, off, n, res, st)
            ev[1].record(st)
            torch.cuda.synchronize()
            times[i].append(ev[0].elapsed_time(ev[1]) / 20)
    for q in ptrs:  # the counter phase: REPS dispatches per buffer, in buffer order
        for _ in range(REPS):
            ctx.classify(q, stride, off, n, res, st)
    torch.cuda.synchronize()
    out = {"frames": n, "reps_per_buffer": REPS,
           "buffers": [{"addr": hex(q), "ms_median": round(statistics.median(t), 5)} for q, t in zip(ptrs, times)]}
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    for q in ptrs:
        hip.hipFree(C.c_void_p(q))


def channels(root):
    """Per-instance counters (rocprofv3 --output-format json: one record per TCC channel x XCC) of each buffer's
    counter-phase dispatches: per pass <root>/<name>/pmc_results.json + <root>/<name>.run.json.  For each buffer:
    the dispatches' median duration under the profiler, the per-instance medians, their spread across the 16
    channels (summed over XCCs) and across all 128 instances."""
    out = {}
    for run_json in sorted(glob.glob(os.path.join(root, "*.run.json"))):
        name = os.path.basename(run_json)[: -len(".run.json")]
        meta = json.load(open(run_json))
        res = glob.glob(os.path.join(root, name, "**", "*results.json"), recursive=True)
        if not res:
            continue
        tool = json.load(open(res[0]))["rocprofiler-sdk-tool"][0]
        names = {k["kernel_id"]: k["kernel_name"] for k in tool["kernel_symbols"]}
        cinfo = {c["id"]["handle"]: c for c in tool["counters"]}
        recs = []
        for r in tool["callback_records"]["counter_collection"]:
            di = r["dispatch_data"]["dispatch_info"]
            if "rx_classify" not in names.get(di["kernel_id"], ""):
                continue
            by_counter = {}
            for x in r["records"]:
                by_counter.setdefault(x["counter_id"]["handle"], []).append(x["value"])
            dur = r["dispatch_data"]["end_timestamp"] - r["dispatch_data"]["start_timestamp"]
            recs.append((di["dispatch_id"], dur, by_counter))
        recs.sort()
        k, reps = len(meta["buffers"]), meta["reps_per_buffer"]
        recs = recs[-k * reps:]
        bufs = []
        for i, b in enumerate(meta["buffers"]):
            rs = recs[i * reps:(i + 1) * reps]
            entry = {**b, "profiled_dispatch_us": round(statistics.median(r[1] for r in rs) / 1e3, 2)}
            for cid, vals in rs[0][2].items():
                cname = cinfo[cid]["name"]
                inst = [statistics.median(r[2][cid][j] for r in rs) for j in range(len(vals))]
                dims = [{d["dimension_name"]: d["index"] for d in x["dimensions"]} for x in cinfo[cid]["instances"]]
                chan = {}
                for v, d in zip(inst, dims):
                    chan[d.get("DIMENSION_INSTANCE", 0)] = chan.get(d.get("DIMENSION_INSTANCE", 0), 0) + v
                cv = [chan[c] for c in sorted(chan)]
                mean_c, mean_i = statistics.mean(cv), statistics.mean(inst)
                entry[cname] = {"total": sum(inst), "per_channel": cv,
                                "channel_max_over_mean": round(max(cv) / mean_c, 4) if mean_c else None,
                                "channel_cv": round(statistics.pstdev(cv) / mean_c, 4) if mean_c else None,
                                "instance_max_over_mean": round(max(inst) / mean_i, 4) if mean_i else None,
                                "instance_cv": round(statistics.pstdev(inst) / mean_i, 4) if mean_i else None}
            bufs.append(entry)
        out[name] = bufs
    print(json.dumps(out, indent=1))


def summarize(root):
    """Per pass directory <root>/<name>/ (rocprofv3 csv) + <root>/<name>.run.json: counters per buffer."""
    out = {}
    for run_json in sorted(glob.glob(os.path.join(root, "*.run.json"))):
        name = os.path.basename(run_json)[: -len(".run.json")]
        meta = json.load(open(run_json))
        rows = []
        for f in glob.glob(os.path.join(root, name, "**", "*counter_collection.csv"), recursive=True):
            rows += [r for r in csv.DictReader(open(f)) if "rx_classify" in r.get("Kernel_Name", "")]
        per = {}
        for r in rows:
            did = int(r.get("Dispatch_Id") or r.get("Correlation_Id"))
            per.setdefault(did, {}).setdefault(r["Counter_Name"], 0.0)
            per[did][r["Counter_Name"]] += float(r["Counter_Value"])
        k, reps = len(meta["buffers"]), meta["reps_per_buffer"]
        dids = sorted(per)[-k * reps:]
        bufs = []
        for i, b in enumerate(meta["buffers"]):
            ds = dids[i * reps:(i + 1) * reps]
            counters = {c: statistics.median(per[d][c] for d in ds) for c in per[ds[0]]}
            bufs.append({**b, **counters})
        out[name] = bufs
    print(json.dumps(out, indent=1))


def orders(out_path, k):
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    n, stride, off = 1 << 20, 2048, 2
    p = pa.rx.GenParams.for_config(2)
    s = pa.gen_frames(p, n, stride, off)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    src = torch.from_numpy(s.reshape(-1)).cuda()
    hip = C.CDLL("libamdhip64.so.7")
    ptrs = []
    for _ in range(k):
        ptr = C.c_void_p()
        assert hip.hipMalloc(C.byref(ptr), C.c_size_t(n * stride)) == 0
        assert hip.hipMemcpy(ptr, C.c_void_p(src.data_ptr()), C.c_size_t(n * stride), 3) == 0
        ptrs.append(ptr.value)
    torch.cuda.synchronize()
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    legs = {"product_xcd_order": lambda q: ctx.classify(q, stride, off, n, res, st),
            "blockidx_order": lambda q: tn.classify_variant(ctx, q, stride, off, n, res, st, 36),
            "no_pipe_stream": lambda q: tn.classify_variant(ctx, q, stride, off, n, res, st, 48),
            "stream_read": lambda q: tn.calib_stream_read(ctx, q, n * stride, sink, st)}
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = [{name: [] for name in legs} for _ in ptrs]
    for _ in range(7):
        for i, q in enumerate(ptrs):
            for name, fn in legs.items():
                fn(q)
                ev[0].record(st)
                for _ in range(10):
                    fn(q)
                ev[1].record(st)
                torch.cuda.synchronize()
                times[i][name].append(ev[0].elapsed_time(ev[1]) / 10)
    out = {"frames": n, "buffers": [{"addr": hex(q), **{name: round(statistics.median(t), 5) for name, t in ts.items()}}
                                    for q, ts in zip(ptrs, times)]}
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


def alloc(out_path, pattern):
    """Buffers allocated in the order `pattern` (t = torch.empty, the bench's way; h = hipMalloc;
    T = torch.from_numpy(host).to("cuda"), exactly bench.py's upload), each filled with the same C2
    frames, then the product kernel timed on each in interleaved rounds: does the allocation path
    or the allocation order decide the slow placement?"""
    import numpy as np
    import torch

    import pollnet_amd as pa

    n, stride, off = 1 << 20, 2048, 2
    p = pa.rx.GenParams.for_config(2)
    s = pa.gen_frames(p, n, stride, off)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    hip = C.CDLL("libamdhip64.so.7")
    bufs, keep = [], []
    src = None
    for kind in pattern:
        if kind == "T":
            b = torch.from_numpy(s.reshape(-1)).to("cuda")
            keep.append(b)
            bufs.append(("T", b.data_ptr()))
        elif kind == "t":
            b = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
            keep.append(b)
            bufs.append(("t", b.data_ptr()))
        else:
            ptr = C.c_void_p()
            assert hip.hipMalloc(C.byref(ptr), C.c_size_t(n * stride)) == 0
            bufs.append(("h", ptr.value))
        if src is None and kind == "T":
            src = keep[-1]
    if src is None:
        src = torch.from_numpy(s.reshape(-1)).to("cuda")
    for kind, q in bufs:
        if q != src.data_ptr():
            assert hip.hipMemcpy(C.c_void_p(q), C.c_void_p(src.data_ptr()), C.c_size_t(n * stride), 3) == 0
    torch.cuda.synchronize()
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    st = torch.cuda.current_stream()
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    times = [[] for _ in bufs]
    for _ in range(7):
        for i, (_, q) in enumerate(bufs):
            ctx.classify(q, stride, off, n, res, st)
            ev[0].record(st)
            for _ in range(10):
                ctx.classify(q, stride, off, n, res, st)
            ev[1].record(st)
            torch.cuda.synchronize()
            times[i].append(ev[0].elapsed_time(ev[1]) / 10)
    out = {"pattern": pattern, "buffers": [{"kind": k, "addr": hex(q), "ms": round(statistics.median(t), 5)}
                                           for (k, q), t in zip(bufs, times)]}
    with open(out_path, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 8)
    elif sys.argv[1] == "alloc":
        alloc(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "orders":
        orders(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 12)
    elif sys.argv[1] == "channels":
        channels(sys.argv[2])
    else:
        summarize(sys.argv[2])
