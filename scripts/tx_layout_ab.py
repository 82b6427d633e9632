#!/usr/bin/env python3
"""pn_tx_fill at frame_off 2 and 14 on the SAME device buffers (same physical HBM), interleaved rounds.

The TX fill's time follows where its frames sit in HBM; comparing the two layouts on separately
allocated buffers mixes placement into the layout effect.  Here 4 rotating buffers are allocated once; each round
copies the offset-2 frames into them (device to device from a staging copy), times the product, then the
offset-14 frames into the same buffers and times again.  Also the two phases alone (tuning variants 13 / 14).

  python3 scripts/tx_layout_ab.py [--rounds 9] [--reps 10]   ->  one JSON object on stdout"""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=9)
    ap.add_argument("--reps", type=int, default=10)
    a = ap.parse_args()
    import numpy as np
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    n, stride, R = 1 << 20, 2048, 4
    p = pa.rx.GenParams.for_config(2)
    st = torch.cuda.current_stream()
    ctx = pa.RxContext(0)
    host = np.empty((n, stride), np.uint8)
    staged = {}
    for off in (2, 14):
        pa.gen_frames(p, n, stride, off, first_index=0, threads=16, out=host)
        d = torch.from_numpy(host.reshape(-1)).cuda()
        v = d.view(n, stride)
        v[:, off + 24:off + 26] = 0x5A
        v[:, off + 50:off + 52] = 0xA5
        staged[off] = d
    bufs = [torch.empty(n * stride, dtype=torch.uint8, device="cuda") for _ in range(R)]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(fn):
        for b in bufs:
            fn(b)
        ev[0].record(st)
        for k in range(a.reps):
            fn(bufs[k % R])
        ev[1].record(st)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / a.reps

    times = {f"{kind}_off{off}": [] for kind in ("product", "phase1_only", "phase2_only") for off in (2, 14)}
    ok = True
    for r in range(a.rounds):
        for off in ((2, 14) if r % 2 == 0 else (14, 2)):
            for b in bufs:
                b.copy_(staged[off])
            ref = staged[off].clone()
            ctx.tx_fill(ref, stride, off, n, None, pa.PN_TX_TCP, st)
            times[f"product_off{off}"].append(timed(lambda d: ctx.tx_fill(d, stride, off, n, None, pa.PN_TX_TCP, st)))
            ok &= bool(torch.equal(bufs[0], ref))
            times[f"phase1_only_off{off}"].append(timed(lambda d: tn.tx_fill_variant(ctx, d, stride, off, n, None, 13, st)))
            times[f"phase2_only_off{off}"].append(timed(lambda d: tn.tx_fill_variant(ctx, d, stride, off, n, None, 14, st)))
    out = {"frames": n, "rotating_buffers": R, "rounds": a.rounds, "same_buffers_for_both_layouts": True,
           "product_frames_equal_reference_fill": ok}
    for k, ts in times.items():
        out[k] = {"ms_median": round(statistics.median(ts), 5), "ms_min": round(min(ts), 5), "ms_max": round(max(ts), 5)}
    out["off14_over_off2"] = round(out["product_off14"]["ms_median"] / out["product_off2"]["ms_median"], 4)
    print(json.dumps(out, indent=1))
    ctx.close()


if __name__ == "__main__":
    main()
