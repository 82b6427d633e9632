#!/usr/bin/env python3
"""Run the TX fill's kernels a few times over rotating resident batches so that
rocprofv3 --pmc can attribute HBM bytes per kernel: pn_tx_fill (tx_fill_kernel +
tx_patch_kernel), phase 2 alone on cold lines (variant 14, needs a TUNING=1 build), and
the calibration stream read of a known byte count (FETCH_SIZE correction).
  rocprofv3 --pmc FETCH_SIZE -d <dir> -- python3 scripts/tx_pmc_probe.py [--frame-off 2]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frame-off", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--reps", type=int, default=6)
    ap.add_argument("--phase2", action="store_true", help="also phase 2 alone (variant 14)")
    a = ap.parse_args()
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    n, off = a.frames, a.frame_off
    p = pa.rx.GenParams.for_config(2)
    s = pa.gen_frames(p, n, 2048, off)
    ctx = pa.RxContext(0)
    bufs = []
    for _ in range(4):
        d = torch.from_numpy(s.reshape(-1)).cuda()
        v = d.view(n, 2048)
        v[:, off + 24:off + 26] = 0x5A
        v[:, off + 50:off + 52] = 0xA5
        bufs.append(d)
    st = torch.cuda.current_stream()
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    for k in range(a.reps):
        ctx.tx_fill(bufs[k % 4], 2048, off, n, None, pa.PN_TX_TCP, st)
    if a.phase2:
        for k in range(a.reps):
            tn.tx_fill_variant(ctx, bufs[k % 4], 2048, off, n, None, 14, st)
    for _ in range(3):
        tn.calib_stream_read(ctx, bufs[0], bufs[0].numel(), sink, st)
    torch.cuda.synchronize()
    print("calib_bytes", bufs[0].numel())


if __name__ == "__main__":
    main()
