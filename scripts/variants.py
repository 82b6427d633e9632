#!/usr/bin/env python3
"""A/B kernel shapes in ONE process, interleaved rounds (guide §5.4 rule 24).
Every variant's records must equal the production kernel's bit for bit."""
import argparse
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

NAMES = {0: "perlane_window", 1: "coop_window", 2: "perlane_defaultpolicy", 3: "coop_defaultpolicy",
         4: "coop_win_default", 5: "coop_store_default", 6: "coop_win_store_default", 7: "coop_store_nt",
         8: "coop_global_store", 9: "coop_tail_masks", 19: "ABL_store8",
         22: "scalar_probe_walk", 23: "grp2_burst_records", 24: "grp4_burst_records", 25: "grp8_burst_records",
         26: "grp16_burst_records", 27: "grp8_records_each", 28: "grp1_lds10k", 29: "grp1_lds14k", 30: "grp8_each_lds10k",
         31: "grp1_vgpr3w", 32: "grp1_vgpr2w", 33: "grp2_burst_vgpr2w", 34: "nopad_5waves", 35: "xcd_contiguous", 36: "blockidx_order", 37: "no_skip_empty_loads", 38: "group_probe", 39: "per_lane_probe", 42: "late_probe", 43: "ABL_home_slot_only", 45: "ABL_home_slot_one_line", 47: "serial_window", 48: "no_pipe_stream",
         11: "ABL_noprobe", 12: "ABL_noreduce", 14: "ABL_nomask", 18: "ABL_nostore", 49: "ABL_store_16KiB", 50: "store_sc0", 55: "ABL_early_store", 51: "store_sc0_nt", 52: "store_sc0_sc1", 53: "store_sc1_nt", 54: "store_sc0_sc1_nt", 56: "grp2_loop_xcd_opaque", 57: "grp4_loop_xcd_opaque", 58: "grp2_loop_xcd", 59: "grp8_loop_xcd_opaque"}
TIMING_ONLY = {11, 12, 14, 18, 19, 43, 45, 49, 55}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--frames", type=int, default=1 << 20)
    ap.add_argument("--rounds", type=int, default=15)
    ap.add_argument("--reps", type=int, default=5)
    ap.add_argument("--variants", default="0,1,2,3,18")
    ap.add_argument("--frame-off", type=int, default=2, help="2 or 18 (the variant kernels are the MIS = 0 class)")
    ap.add_argument("--uncached", action="store_true", help="frame ring from hipExtMallocWithFlags(Uncached)")
    a = ap.parse_args()
    import numpy as np
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    p = pa.rx.GenParams.for_config(a.config)
    s = pa.gen_frames(p, a.frames, 2048, a.frame_off)
    t = pa.gen_conn_table(p)
    wire = pa.wire_bytes(s, 2048, a.frame_off, a.frames)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(t)
    frames = torch.from_numpy(s.reshape(-1)).cuda()
    if a.uncached:
        import ctypes as C
        hip = C.CDLL("libamdhip64.so.7")
        ptr = C.c_void_p()
        assert hip.hipExtMallocWithFlags(C.byref(ptr), C.c_size_t(frames.numel()), C.c_uint(0x3)) == 0  # Uncached
        assert hip.hipMemcpy(ptr, C.c_void_p(frames.data_ptr()), C.c_size_t(frames.numel()), 3) == 0  # D2D

        class Raw:  # minimal stand-in exposing data_ptr/numel for the bindings
            def __init__(self, p, n):
                self.p, self.n = p, n

            def data_ptr(self):
                return self.p

            def numel(self):
                return self.n

        frames = Raw(ptr.value, frames.numel())
    ref = torch.empty(a.frames * 16, dtype=torch.uint8, device="cuda")
    res = torch.empty_like(ref)
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    st = torch.cuda.current_stream()
    ctx.classify(frames, 2048, a.frame_off, a.frames, ref, st)
    vs = [int(x) for x in a.variants.split(",")]
    for v in vs:
        res.zero_()
        tn.classify_variant(ctx, frames, 2048, a.frame_off, a.frames, res, st, v)
        torch.cuda.synchronize()
        if v not in TIMING_ONLY:
            assert torch.equal(res, ref), f"variant {v} differs from production"
    times = {v: [] for v in vs}
    times["calib"] = []
    SLOT_MODES = [(1536, 0), (1536, 16), (1536, 8)]  # (bytes per slot, record store bytes)
    for b, wpg in SLOT_MODES:
        times[f"slotread_{b}_store{wpg}"] = []
    times["prod"] = []
    times["prod_b2b50"] = []
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]

    def timed(fn):
        for _ in range(2):
            fn()
        ev[0].record(st)
        for _ in range(a.reps):
            fn()
        ev[1].record(st)
        torch.cuda.synchronize()
        return ev[0].elapsed_time(ev[1]) / a.reps

    for _ in range(a.rounds):
        times["calib"].append(timed(lambda: tn.calib_stream_read(ctx, frames, frames.numel(), sink, st)))
        for b, wpg in SLOT_MODES:
            tgt = res if wpg else sink
            times[f"slotread_{b}_store{wpg}"].append(timed(lambda: tn.calib_slot_read(ctx, frames, a.frames, 2048, b, tgt, st, wpg)))
        times["prod"].append(timed(lambda: ctx.classify(frames, 2048, a.frame_off, a.frames, res, st)))
        r0 = a.reps
        a.reps = 50
        times["prod_b2b50"].append(timed(lambda: ctx.classify(frames, 2048, a.frame_off, a.frames, res, st)))
        a.reps = r0
        for v in vs:
            times[v].append(timed(lambda: tn.classify_variant(ctx, frames, 2048, a.frame_off, a.frames, res, st, v)))
    algo = wire + 16 * a.frames
    out = {"config": a.config, "frames": a.frames,
           "calib_stream_read_tbps": round(frames.numel() / (statistics.median(times["calib"]) * 1e-3) / 1e12, 3)}
    for k, ts in times.items():
        if k == "calib":
            continue
        med = statistics.median(ts)
        if isinstance(k, str) and k.startswith("slotread_"):
            b = int(k.split("_")[1])
            out[k] = {"ms_median": round(med, 4), "read_tbps": round(b * a.frames / (med * 1e-3) / 1e12, 3)}
            continue
        out[NAMES.get(k, k)] = {"ms_median": round(med, 4), "ms_min": round(min(ts), 4),
                               "algo_tbps": round(algo / (med * 1e-3) / 1e12, 3)}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
