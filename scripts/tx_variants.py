#!/usr/bin/env python3
"""A/B of pn_tx_fill shapes in ONE process, interleaved rounds (TCP mode, C2 frames).
Every variant's filled frames must equal the production fill's byte for byte (except
the timing-only ablation 9).  Also times the RX classify kernel over the same frames
and the no-arithmetic slot-read ceilings for reference."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {0: "inplace_u16_stores", 2: "inplace_tile_wb128_sc1", 9: "ABL_nowrite",
         10: "twophase_line0_nt", 11: "twophase_blockidx_order", 13: "phase1_only", 14: "phase2_only",
         15: "phase1_rec16_global", 16: "phase1_rec16_buffer_sc1", 17: "inplace_u16_line0_default",
         18: "inplace_tile_wb128_line0_default", 19: "inplace_tile_wb128_sc1_line0_default",
         20: "twophase_4waves", 21: "twophase_xcd_order", 30: "phase2_u16_nt",
         32: "phase2_sector_plain", 33: "phase2_sector_nt",
         35: "PROBE_full64B_write_nofetch", 36: "PROBE_full128B_write_nofetch", 40: "product_shape_twophase",
         41: "product_shape_inplace", 42: "product_shape_twophase_skip_empty_loads",
         43: "product_shape_twophase_concurrent_window", 50: "product_shape_phase2_u16_writethrough",
         51: "product_shape_phase2_sector64_writethrough", 52: "product_shape_phase2_then_l2_release"}
TIMING_ONLY = {9, 13, 14, 15, 16, 35, 36}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=12)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--frame-off", type=int, default=2)
    ap.add_argument("--variants", default="0,2,9,10,11,13,14")
    ap.add_argument("--rotate", type=int, default=1, help="distinct frame buffers the timed calls rotate over")
    a = ap.parse_args()
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    n, off = a.frames, a.frame_off
    p = pa.rx.GenParams.for_config(2)
    s = pa.gen_frames(p, n, 2048, off)
    t = pa.gen_conn_table(p)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(t)
    base = torch.from_numpy(s.reshape(-1)).cuda()
    v = base.view(n, 2048)
    v[:, off + 24:off + 26] = 0x5A
    v[:, off + 50:off + 52] = 0xA5
    st = torch.cuda.current_stream()
    ref = base.clone()
    ctx.tx_fill(ref, 2048, off, n, None, pa.PN_TX_TCP, st)
    work = base.clone()
    vs = [int(x) for x in a.variants.split(",")]
    arg = lambda var: None  # noqa: E731
    for var in vs:
        if var in (35, 36):
            continue  # write probes: garbage into the frames
        work.copy_(base)
        if var == 14:
            tn.tx_fill_variant(ctx, work, 2048, off, n, None, 13, st)  # phase 2 needs phase 1's records
        tn.tx_fill_variant(ctx, work, 2048, off, n, arg(var), var, st)
        torch.cuda.synchronize()
        if var not in TIMING_ONLY or var == 14:
            assert torch.equal(work, ref), f"variant {var} differs from production"
    works = [work] + [base.clone() for _ in range(max(1, a.rotate) - 1)]
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    R = len(works)
    probe_bufs = [base.clone() for _ in range(R)] if any(v in (35, 36) for v in vs) else []

    def timed_on(bufs, fn):  # fn(buffer): the calls rotate over the frame buffers
        for b in bufs:
            fn(b)
        ev[0].record(st)
        for k in range(a.reps):
            fn(bufs[k % len(bufs)])
        ev[1].record(st)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / a.reps

    def timed(fn):
        return timed_on(works, fn)

    times = {var: [] for var in vs}
    times["prod"], times["rx_classify"], times["slotread_1536"], times["slotread_1536_store16"] = [], [], [], []
    for _ in range(a.rounds):
        times["prod"].append(timed(lambda w: ctx.tx_fill(w, 2048, off, n, None, pa.PN_TX_TCP, st)))
        times["rx_classify"].append(timed(lambda w: ctx.classify(w, 2048, off, n, res, st)))
        if off == 2:
            times["slotread_1536"].append(timed(lambda w: tn.calib_slot_read(ctx, w, n, 2048, 1536, sink, st, 0)))
            times["slotread_1536_store16"].append(timed(lambda w: tn.calib_slot_read(ctx, w, n, 2048, 1536, res, st, 16)))
        for var in vs:
            if var in (35, 36):  # the write probes scribble on the frames: give them their own buffers
                times[var].append(timed_on(probe_bufs, lambda w: tn.tx_fill_variant(ctx, w, 2048, off, n, None, var, st)))
            else:
                times[var].append(timed(lambda w: tn.tx_fill_variant(ctx, w, 2048, off, n, arg(var), var, st)))
    algo = 1504 * n
    out = {"frames": n, "frame_off": off, "algo_bytes_per_frame": 1504, "rotating_buffers": R}
    for k, ts in times.items():
        if not ts:
            continue
        med = statistics.median(ts)
        out[NAMES.get(k, k)] = {"ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                               "algo_tbps": round(algo / (med * 1e-3) / 1e12, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
