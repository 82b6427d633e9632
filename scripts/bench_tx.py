#!/usr/bin/env python3
"""TX checksum fill (pn_tx_fill) on one MI355X, device-resident.

One step = one pn_tx_fill launch over a batch of outgoing frames already in HBM: the
IP and TCP checksums of every frame recomputed from its bytes and written in place
(PN_TX_TCP), the values efvitcp's incremental send path (sendBuf + setOptDataLen,
TcpConn.h:310-323, Core.h:157-163) writes.  Workload: the C2 generator's 1514-B
frames (tot_len 1500) with both checksum fields scrambled, rotating over --batches
distinct resident batches.  Layouts: the RX ring layout (2048-B slots, frame_off 2:
cooperative line-0 window) and efvitcp's SendBuf layout (frame_off 14 =
offsetof(SendBuf, eth_hdr), Core.h:147-156; per-lane window).

Algorithmic bytes per frame = tot_len read (IP header + segment: all a checksum needs)
+ 4 B written (+ 2 B lens read and 2 B tot_len written with --lens).

Prints one JSON line per layout.  CPU baseline beside it (rank-0 host, bounded sample):
orc_tx_fill_batch (the same recomputation, "port") on 16 threads and 1 thread, and the
reference's own per-segment work, copyAndSum into a send buffer + setOptDataLen
(orc_tx_copy_and_sum_batch), 1 thread.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBS = 8000.0
STRIDE = 2048


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--batches", type=int, default=4)
    ap.add_argument("--frame-offs", default="2,14")
    ap.add_argument("--lens", action="store_true", help="also set tot_len from a lens array (setOptDataLen)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()

    import torch

    import pollnet_amd as pa
    from oracle import pyoracle as orc

    n, R = args.frames, max(1, args.batches)
    ctx = pa.RxContext(0)
    p = pa.rx.GenParams.for_config(2)
    host = np.empty((n, STRIDE), dtype=np.uint8)
    lines = []
    for off in [int(x) for x in args.frame_offs.split(",")]:
        batches, exp0 = [], None
        for b in range(R):
            pa.gen_frames(p, n, STRIDE, off, first_index=b * n, threads=16, out=host)
            if b == 0:
                exp0 = host[:4096].copy()
            d = torch.from_numpy(host.reshape(-1)).cuda()
            v = d.view(n, STRIDE)
            v[:, off + 24:off + 26] = 0x5A  # ip checksum
            v[:, off + 50:off + 52] = 0xA5  # tcp checksum
            batches.append(d)
        tot = 1500
        lens = torch.full((n,), tot - 40, dtype=torch.int16, device="cuda") if args.lens else None
        stream = torch.cuda.current_stream()
        # correctness gate: batch 0's first 4096 frames after the fill vs the oracle's recomputation
        ctx.tx_fill(batches[0], STRIDE, off, n, lens, pa.PN_TX_TCP, stream)
        torch.cuda.synchronize()
        got = batches[0][: 4096 * STRIDE].cpu().numpy().reshape(4096, STRIDE)
        exp = exp0.copy()
        exp[:, off + 24:off + 26] = 0x5A
        exp[:, off + 50:off + 52] = 0xA5
        orc.tx_fill_batch(exp, STRIDE, off, 4096, None, orc.TX_TCP)
        verified = bool(np.array_equal(got, exp))
        for w in range(args.warmup):
            ctx.tx_fill(batches[w % R], STRIDE, off, n, lens, pa.PN_TX_TCP, stream)
        torch.cuda.synchronize()
        ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0 = time.perf_counter()
        ev0.record(stream)
        for k in range(args.steps):
            ctx.tx_fill(batches[k % R], STRIDE, off, n, lens, pa.PN_TX_TCP, stream)
        ev1.record(stream)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t0
        kern_ms = ev0.elapsed_time(ev1) / args.steps
        per_frame = tot + 4 + (4 if args.lens else 0)
        algo = per_frame * n
        achieved = algo / (kern_ms * 1e-3) / 1e9
        wire = (14 + tot) * n
        line = {
            "metric": "TX checksum fill, device-resident Gbit/s of 1514-B frames (pn_tx_fill, PN_TX_TCP)",
            "value": round(wire * 8 * args.steps / wall / 1e9, 2),
            "unit": "Gbit/s",
            "mframes_per_s": round(n * args.steps / wall / 1e6, 2),
            "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(wall * 1e3 / args.steps, 4),
            "dtype": "u16/u32 integer (one's-complement sums)",
            "config": {"workload": "C2 frames (tot_len 1500), both checksums scrambled", "frames": n,
                       "slot_stride": STRIDE, "frame_off": off, "lens": bool(args.lens),
                       "resident_batches": R},
            "verified_vs_oracle": verified,
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
                         "kernel": "tx_fill_kernel + tx_patch_kernel (one pn_tx_fill call)", "kernel_ms_avg": round(kern_ms, 5),
                         "algorithmic_bytes_per_launch": algo, "bytes_per_frame": per_frame},
        }
        del batches
        torch.cuda.empty_cache()
        lines.append(line)

    if not args.no_cpu_baseline:
        sample = min(n, 1 << 17)
        pa.gen_frames(p, sample, STRIDE, 2, threads=16, out=host[:sample])
        slots = host[:sample]
        out = np.empty_like(slots)

        def rate(fn, secs):
            t0, k = time.perf_counter(), 0
            while True:
                fn()
                k += 1
                el = time.perf_counter() - t0
                if el >= secs:
                    return k * sample / el

        thr = max(1, min(16, os.cpu_count() or 1))
        f_mt = rate(lambda: orc.tx_fill_batch(slots, STRIDE, 2, sample, None, orc.TX_TCP, thr), args.cpu_seconds * 0.4)
        f_1 = rate(lambda: orc.tx_fill_batch(slots, STRIDE, 2, sample, None, orc.TX_TCP, 1), args.cpu_seconds * 0.3)
        f_cas = rate(lambda: orc.tx_copy_and_sum_batch(slots, out, STRIDE, 2, sample, 1), args.cpu_seconds * 0.3)
        g = lambda fr: round(fr * 1514 * 8 / 1e9, 2)  # noqa: E731
        cpu = {"value": g(f_mt), "unit": "Gbit/s", "cores": thr, "kind": "port",
               "sample": f"orc_tx_fill_batch (the same recomputation from the bytes, oracle/pn_tx_oracle.c -O3) over "
                         f"{sample} C2 frames",
               "mframes_per_s": round(f_mt / 1e6, 3),
               "single_thread": {"value": g(f_1), "mframes_per_s": round(f_1 / 1e6, 3), "cores": 1},
               "reference_copy_and_sum_1t": {"value": g(f_cas), "mframes_per_s": round(f_cas / 1e6, 3), "cores": 1,
                                             "note": "copyAndSum of each segment into a send buffer + "
                                                     "setOptDataLen (TcpConn.h:257-299, Core.h:157-163)"}}
        for line in lines:
            line["cpu_baseline"] = cpu
    for line in lines:
        print(json.dumps(line), flush=True)
    ctx.close()


if __name__ == "__main__":
    main()
