#!/usr/bin/env python3
"""Benchmark: efvitcp RX per-frame transform on MI355X (device-resident).

One step = one pn_classify launch over this rank's batch of RX-ring slots already
resident in HBM (parse + IP/TCP checksum verification + conn-table probe +
payload off/len, one 16-B record per frame).  Default workload = BASELINE config
C2 (1 Mi x 1514-B IPv4/TCP frames, 1 flow) per GPU; N GPUs = N independent
contiguous index shards of one global batch (weak scaling, no collective on the
data path — torch.distributed is used only for the start barrier and the
max-over-ranks time).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--config 2|3|4|5] [--frames N]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...

Rank 0 prints ONE JSON line (metric = wire Gbit/s = 8*sum(14+tot_len)/t, plus
Mframes/s, the roofline of the kernel, the CPU baseline and the pinned-host
end-to-end rate).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
STRIDE, FRAME_OFF = 2048, 2  # RecvBufSize (Core.h:45); IP header 16-B aligned

WORKLOADS = {
    2: "C2: 1514-B IPv4/TCP frames (tot_len 1500), 1 flow, 2048-B slots",
    3: "C3: 64-1514-B mixed frames, 1024 flows (32 TIME_WAIT, 1/64 miss), 2048-B slots",
    4: "C4: 1514-B frames over 1024 flows, 2048-B slots (16 Mi frames over 8 GPUs)",
    5: "C5: IPv4 options + odd lengths + bad-checksum + adversarial probe cluster, 2048-B slots",
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--frames", type=int, default=0, help="frames per GPU (default: 1 Mi; C4: 2 Mi)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="budget for the CPU baseline leg")
    ap.add_argument("--batches", type=int, default=4,
                    help="distinct resident batches the steps rotate over (defeats reuse of a fixed slice of "
                         "the 256 MiB memory-side cache across launches)")
    return ap.parse_args()


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(slots, n, entries, mask, max_conn, budget_s):
    """The oracle (a C port of the reference path, "port") on this host's cores:
    'ref parse + checksum' (Core::checksum + pollNet + onPack header, Core.h:448-526,
    TcpConn.h:469-473), all cores and 1 thread, plus the release path (no checksum)."""
    from oracle import pyoracle as orc

    threads = max(1, min(16, os.cpu_count() or 1))
    sample = min(n, 1 << 18)  # 256 Ki frames (~0.4 GB of frame bytes)
    import pollnet_amd as pa

    wire = pa.wire_bytes(slots, STRIDE, FRAME_OFF, sample)

    def rate(fn_threads, release, secs):
        t0 = time.perf_counter()
        passes = 0
        while True:
            orc.classify_batch(slots, STRIDE, FRAME_OFF, sample, entries, mask, max_conn, threads=fn_threads,
                               release=release, ref_only=not release)
            passes += 1
            el = time.perf_counter() - t0
            if el >= secs:
                return passes * sample / el, passes * wire * 8 / el / 1e9, passes

    c1 = c1_socket_loopback()
    fr_mt, gb_mt, p_mt = rate(threads, False, budget_s * 0.5)
    fr_1, gb_1, p_1 = rate(1, False, budget_s * 0.3)
    fr_rel, gb_rel, _ = rate(1, True, budget_s * 0.2)
    return {
        "value": round(gb_mt, 2),
        "unit": "Gbit/s",
        "cores": threads,
        "kind": "port",
        "sample": f"'ref parse + checksum' (orc_refsum_batch: Core::checksum + pollNet + onPack header) over "
                  f"{sample} frames of the same workload, {p_mt} passes; oracle/pn_oracle.c -O3 -march=x86-64-v3, "
                  f"contiguous index shards over {threads} threads",
        "mframes_per_s": round(fr_mt / 1e6, 3),
        "single_thread": {"value": round(gb_1, 2), "unit": "Gbit/s", "mframes_per_s": round(fr_1 / 1e6, 3),
                          "cores": 1},
        "release_path_no_checksum_1t": {"value": round(gb_rel, 2), "unit": "Gbit/s",
                                        "mframes_per_s": round(fr_rel / 1e6, 3), "cores": 1},
        "host_cpu": _cpu_model(),
        "c1_socket_loopback_ref": c1,
    }


def c1_socket_loopback(seconds=1.5):
    """BASELINE config C1 beside it: the reference's own Socket.h server + client
    (oracle/_ref/ref_socket_c1, built from /root/reference by oracle/ref.mk) echoing
    1500-B messages over 127.0.0.1, window 1 (ping-pong RTT) and 8."""
    import subprocess

    exe = os.path.join(ROOT, "oracle", "_ref", "ref_socket_c1")
    if not os.path.exists(exe):
        return {"error": "oracle/_ref/ref_socket_c1 not built"}
    out = {}
    for w, port in ((1, 23411), (8, 23412)):
        try:
            r = subprocess.run([exe, str(seconds), str(w), str(port)], capture_output=True, text=True, timeout=30)
            out[f"window_{w}"] = json.loads(r.stdout.strip().splitlines()[-1])
        except Exception as ex:  # measured extra; never blocks the bench line
            out[f"window_{w}"] = {"error": str(ex)}
    return out


def _cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def e2e_rate(torch, ctx, slots, n, chunk=1 << 16, passes=3, stride=STRIDE):
    """Host ring -> GPU -> host records: pinned H2D of each chunk, kernel, D2H of
    its records, double-buffered over 2 streams (copy/compute overlap).  stride < 2048:
    the same frames re-laid in tighter slots (less PCIe per frame)."""
    import pollnet_amd as pa

    nchunks = (n + chunk - 1) // chunk
    if stride != STRIDE:  # the 1514-B frames of the 2-KiB slots re-laid at `stride` (pad byte included)
        slots = np.ascontiguousarray(slots[:n, :stride])
    host = torch.from_numpy(slots.reshape(-1)[: n * stride]).pin_memory()
    host_res = torch.empty(n * 16, dtype=torch.uint8).pin_memory()
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    dev = [torch.empty(chunk * stride, dtype=torch.uint8, device="cuda") for _ in range(2)]
    dres = [torch.empty(chunk * 16, dtype=torch.uint8, device="cuda") for _ in range(2)]
    torch.cuda.synchronize()
    best = None
    for _ in range(passes):
        t0 = time.perf_counter()
        for c in range(nchunks):
            b = c & 1
            s = streams[b]
            lo = c * chunk
            m = min(chunk, n - lo)
            with torch.cuda.stream(s):
                dev[b][: m * stride].copy_(host[lo * stride:(lo + m) * stride], non_blocking=True)
                ctx.classify(dev[b], stride, FRAME_OFF, m, dres[b], s)
                host_res[lo * 16:(lo + m) * 16].copy_(dres[b][: m * 16], non_blocking=True)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    wire = pa.wire_bytes(slots, stride, FRAME_OFF, n)
    return {"gbit_per_s": round(wire * 8 / best / 1e9, 2), "mframes_per_s": round(n / best / 1e6, 3),
            "h2d_gb_per_s": round(n * stride / best / 1e9, 2), "chunk_frames": chunk,
            "note": f"pinned hipMemcpyAsync H2D of whole {stride}-B slots + kernel + D2H records, 2 streams"}, host_res


def e2e_zero_copy(torch, ctx, slots, n, passes=3):
    """Host ring in place: the kernel reads the pinned host slots over PCIe (only each frame's
    lines cross the link) and writes the records into pinned host memory; one launch per pass."""
    import pollnet_amd as pa

    host = torch.from_numpy(slots.reshape(-1)[: n * STRIDE]).pin_memory()
    host_res = torch.empty(n * 16, dtype=torch.uint8).pin_memory()
    stream = torch.cuda.current_stream()
    ctx.classify(host, STRIDE, FRAME_OFF, n, host_res, stream)
    torch.cuda.synchronize()
    best = None
    for _ in range(passes):
        t0 = time.perf_counter()
        ctx.classify(host, STRIDE, FRAME_OFF, n, host_res, stream)
        torch.cuda.synchronize()
        el = time.perf_counter() - t0
        best = el if best is None else min(best, el)
    wire = pa.wire_bytes(slots, STRIDE, FRAME_OFF, n)
    return {"gbit_per_s": round(wire * 8 / best / 1e9, 2), "mframes_per_s": round(n / best / 1e6, 3),
            "note": "pn_classify on pinned host 2048-B slots (zero copy), records to pinned host memory"}, host_res


def ceilings(torch, ctx, frames, n, res, stream, slot_pattern, lens=None, reps=10):
    """Same-run bandwidth ceilings (no arithmetic): a front-to-back stream read of the
    whole ring, and the RX kernel's own load pattern over the first 1536 B of each slot
    with and without its 16-B/frame record writes.  With `lens` (u32 per slot: slot start
    to the frame's pad byte), the same pattern over each frame's own lines, in the RX
    kernel's workgroup order and occupancy: the ceiling for mixed-size rings (C3/C5)."""
    from pollnet_amd import tuning as tn  # measurement-only library, never the product path

    sink = torch.zeros(4096, dtype=torch.int32, device=frames.device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def t(fn):
        fn()
        ev[0].record(stream)
        for _ in range(reps):
            fn()
        ev[1].record(stream)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / reps * 1e-3

    ts = t(lambda: tn.calib_stream_read(ctx, frames, frames.numel(), sink, stream))
    out = {"stream_read_gbs": round(frames.numel() / ts / 1e9, 1),
           "note": "calib kernels in pollnet_amd/csrc/rx_tuning.hip (libpollnet_amd_tuning.so); no header work, no arithmetic"}
    if slot_pattern:
        t0 = t(lambda: tn.calib_slot_read(ctx, frames, n, STRIDE, 1536, sink, stream, 0))
        t16 = t(lambda: tn.calib_slot_read(ctx, frames, n, STRIDE, 1536, res, stream, 16))
        out["slot_pattern_read_gbs"] = round(n * 1536 / t0 / 1e9, 1)
        out["slot_pattern_read_plus_16B_records_ms"] = round(t16 * 1e3, 5)
    if lens is not None:
        lens_dev = torch.from_numpy(lens).to(frames.device)
        tv0 = t(lambda: tn.calib_slot_read_var(ctx, frames, n, STRIDE, lens_dev, sink, stream, 0))
        tv16 = t(lambda: tn.calib_slot_read_var(ctx, frames, n, STRIDE, lens_dev, res, stream, 16))
        out["frame_lines_read_ms"] = round(tv0 * 1e3, 5)
        out["frame_lines_read_plus_16B_records_ms"] = round(tv16 * 1e3, 5)
    return out


def load_pmc_traffic(workload_key):
    """HBM bytes per launch from the committed rocprofv3 --pmc summary (profiles/)."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        e = d.get(workload_key)
        return None if e is None else e.get("hbm_bytes_per_launch")
    except (OSError, ValueError):
        return None


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import pollnet_amd as pa
    from pollnet_amd.shard import shard_range

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE")
    # PN_BENCH_DIST_BACKEND=gloo rehearses the N>1 flow with several ranks on one GPU (the timing reduction
    # then runs on CPU tensors); the measured runs use nccl (= RCCL), one rank per GPU
    backend = os.environ.get("PN_BENCH_DIST_BACKEND", "nccl")
    dev = local_rank if backend == "nccl" else local_rank % max(1, torch.cuda.device_count())
    red_dev = f"cuda:{dev}" if backend == "nccl" else "cpu"
    torch.cuda.set_device(dev)
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)

    cfg = args.config
    n = args.frames or ((1 << 21) if cfg == 4 else (1 << 20))
    params = pa.rx.GenParams.for_config(cfg)
    lo, _ = shard_range(rank, world, n)
    local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(world)))
    gen_threads = max(1, min(16, (os.cpu_count() or 16) // max(1, local_world)))
    t0 = time.perf_counter()
    R = max(1, args.batches)
    table = pa.gen_conn_table(params)
    entries, mask = table.snapshot()
    ctx = pa.RxContext(dev)
    ctx.set_conn_table(table)
    # R distinct batches per rank; batch b of rank r holds global frames [(b*world + r)*n, +n)
    frames_b, wires = [], []
    host = np.empty((n, STRIDE), dtype=np.uint8)
    slots = None
    for b in range(R):
        first = (b * world + rank) * n if R > 1 else lo
        pa.gen_frames(params, n, STRIDE, FRAME_OFF, first_index=first, threads=gen_threads, out=host)
        wires.append(pa.wire_bytes(host, STRIDE, FRAME_OFF, n))
        frames_b.append(torch.from_numpy(host.reshape(-1)).to(f"cuda:{dev}"))
        if b == 0:
            slots = host.copy()  # batch 0 stays on the host: oracle check, CPU baseline, e2e leg
    del host
    wire = wires[0]
    frames = frames_b[0]
    log(f"[rank {rank}] generated {R} x {n} frames ({sum(wires) / 1e9:.2f} GB wire) in {time.perf_counter() - t0:.1f}s")

    res = torch.empty(n * 16, dtype=torch.uint8, device=f"cuda:{dev}")
    stream = torch.cuda.current_stream()

    # correctness gate on the measured configuration: first 4096 records vs the oracle
    ctx.classify(frames, STRIDE, FRAME_OFF, n, res, stream)
    torch.cuda.synchronize()
    verified = None
    if rank == 0:
        from oracle import pyoracle as orc

        k = min(n, 4096)
        exp = orc.classify_batch(slots, STRIDE, FRAME_OFF, k, entries, mask, table.max_conn_cnt, threads=8)
        got = res[: k * 16].cpu().numpy().view(pa.RESULT_DTYPE)
        verified = bool(np.array_equal(got, exp))
        if not verified:
            log("ERROR: GPU records differ from the oracle on the bench batch")

    for w in range(args.warmup):
        ctx.classify(frames_b[w % R], STRIDE, FRAME_OFF, n, res, stream)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for k in range(args.steps):
        ctx.classify(frames_b[k % R], STRIDE, FRAME_OFF, n, res, stream)
    ev1.record(stream)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if world > 1:
        dist.barrier()
    wall = t1 - t0
    kern_ms = ev0.elapsed_time(ev1) / args.steps
    if world > 1:
        tt = torch.tensor([wall, kern_ms], dtype=torch.float64, device=red_dev)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        wall, kern_ms_max = float(tt[0]), float(tt[1])
    else:
        kern_ms_max = kern_ms

    total_frames = n * world * args.steps
    step_wire = float(sum(wires[k % R] for k in range(args.steps)))  # this rank's wire bytes over the K steps
    total_wire = step_wire
    if world > 1:
        wt = torch.tensor([step_wire], dtype=torch.float64, device=red_dev)
        dist.all_reduce(wt, op=dist.ReduceOp.SUM)
        total_wire = float(wt[0])
    gbit = total_wire * 8 / wall / 1e9
    mfps = total_frames / wall / 1e6

    out = None
    if rank == 0:
        # every frame byte read once + the 16-B record written, averaged over the launches timed
        algo_bytes = int(step_wire / args.steps) + 16 * n
        achieved = algo_bytes / (kern_ms * 1e-3) / 1e9
        wl_key = f"c{cfg}_n{n}"
        traffic = load_pmc_traffic(wl_key)
        out = {
            "metric": "device-resident Gbit/s + Mframes/s, 1500 B IPv4/TCP frames, 1/2/4/8 MI355X",
            "value": round(gbit, 2),
            "unit": "Gbit/s",
            "mframes_per_s": round(mfps, 2),
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(wall * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u16/u32 integer (one's-complement sums)",
            "data": "synthetic (deterministic seeded generator, pollnet_amd/csrc/framegen.cpp)",
            "config": {"workload": WORKLOADS[cfg], "frames_per_gpu": n, "slot_stride": STRIDE, "frame_off": FRAME_OFF,
                       "parallelism": f"index-sharded x{world}, no collective", "global_frames": n * world,
                       "resident_batches_per_gpu": R},
            "verified_vs_oracle": verified,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic,
                         "kernel": "rx_classify_kernel", "kernel_ms_avg": round(kern_ms, 5),
                         "kernel_ms_avg_max_over_ranks": round(kern_ms_max, 5),
                         "algorithmic_bytes_per_launch": algo_bytes,
                         "bytes_per_frame": round(algo_bytes / n, 2)},
        }
    if rank == 0 and world == 1:  # the slot-pattern ceilings are for 1514-B frames (1536 B of lines per slot)
        tl = slots[:, FRAME_OFF + 16].astype(np.uint32) << 8 | slots[:, FRAME_OFF + 17]  # ip tot_len (BE)
        lens = (FRAME_OFF + 14 + tl + (tl & 1)).astype(np.uint32)  # through the pad byte of odd segments
        c = ceilings(torch, ctx, frames, n, res, stream, slot_pattern=cfg in (2, 4), lens=lens)
        if cfg in (2, 4):
            c["kernel_vs_read_plus_records_ceiling"] = round(c["slot_pattern_read_plus_16B_records_ms"] / kern_ms, 4)
        c["kernel_vs_frame_lines_ceiling"] = round(c["frame_lines_read_plus_16B_records_ms"] / kern_ms, 4)
        out["roofline"]["same_run_ceilings"] = c
    if rank == 0 and world == 1 and not args.no_e2e:
        try:
            out["e2e_pinned_host"], _ = e2e_rate(torch, ctx, slots, n)
            if cfg in (2, 4):  # 1514-B frames + pad byte fit 1536-B slots: 25 % less PCIe per frame
                out["e2e_pinned_host_1536B_slots"], _ = e2e_rate(torch, ctx, slots, n, stride=1536)
            out["e2e_zero_copy_pinned_host"], zres = e2e_zero_copy(torch, ctx, slots, n)
            ctx.classify(frames, STRIDE, FRAME_OFF, n, res, stream)  # batch 0 resident, as the zero-copy run read it
            torch.cuda.synchronize()
            if not torch.equal(zres, res.cpu()):
                out["e2e_zero_copy_pinned_host"]["error"] = "records differ from the device-resident run"
        except Exception as ex:  # measured extra; never blocks the bench line
            out["e2e_pinned_host"] = {"error": str(ex)}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(slots, n, entries, mask, table.max_conn_cnt, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(out), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
