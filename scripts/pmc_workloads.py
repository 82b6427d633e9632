#!/usr/bin/env python3
"""The bench's workloads, one after another in one process, for rocprofv3 --pmc passes (scripts/pmc_refresh.sh).

Every launch of a pollnet kernel goes through call(label, kernels, fn), which records the label and the kernel
families it dispatches, in order; scripts/pmc_refresh.py matches that sequence to the dispatches in the pass's
counter CSV (Dispatch_Id order) and turns each label's per-call counters into the entries of
profiles/pmc_traffic.json.  The workloads are bench.py's (same generators, strides, rotating resident batches);
every batch is gated against the committed digests (or the oracle) so the counters are of a correct run.

  python3 scripts/pmc_workloads.py --out DIR [--uncached] [--only LABEL,...] [--tx-variants V,...]

--uncached adds the round-5 experiment: the C2 ring in uncached device memory
(hipExtMallocWithFlags(hipDeviceMallocUncached)), pn_match_streams and the release-path classify on it, records
compared with the same calls on ordinary memory.  --tx-variants adds the TX fill's tuning variants (the
measurement-only library, scripts/tx_variants.py's numbering) at both layouts, labels x_tx_v<V>/frame_off_<off>:
experiments, kept out of profiles/pmc_traffic.json by the summariser."""
import argparse
import ctypes
import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

STRIDE, FRAME_OFF = 2048, 2
N = 1 << 20
CALLS = 12  # measured calls per workload (after 4 warm ones)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Seq:
    def __init__(self):
        self.calls = []  # [label, [kernel families]]

    def call(self, label, kernels, fn):
        self.calls.append([label, list(kernels)])
        fn()


def lib_sha():
    with open(os.path.join(ROOT, "pollnet_amd", "libpollnet_amd.so"), "rb") as f:
        return hashlib.sha256(f.read()).hexdigest()


def golden(cfg, first, n):
    with open(os.path.join(ROOT, "tests", "golden", "full_digests.json")) as f:
        full = json.load(f)
    cands = [dict(full[f"c{cfg}"], first_index=0)] if f"c{cfg}" in full else []
    cands += full.get(f"c{cfg}_shards", [])
    for d in cands:
        if d.get("first_index", 0) == first and d["n"] == n:
            return d["records_sha256"]
    return None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", required=True)
    ap.add_argument("--uncached", action="store_true")
    ap.add_argument("--only", default="")
    ap.add_argument("--tx-variants", default="")
    args = ap.parse_args()
    only = set(filter(None, args.only.split(",")))
    import torch

    import pollnet_amd as pa
    from pollnet_amd import tuning as tn

    want = lambda label: not only or label in only  # noqa: E731
    dev = torch.cuda.current_device()
    stream = torch.cuda.current_stream()
    seq = Seq()
    plan = {"lib_sha256": lib_sha(), "frames": N, "workloads": {}, "gates": {}}
    host = np.empty((N, STRIDE), dtype=np.uint8)

    def batches(cfg, count, first_of, off=FRAME_OFF, n=N, hbuf=None):
        p = pa.rx.GenParams.for_config(cfg)
        hb = host if hbuf is None else hbuf
        out, wires = [], []
        for b in range(count):
            pa.gen_frames(p, n, STRIDE, off, first_index=first_of(b), threads=16, out=hb)
            wires.append(pa.wire_bytes(hb, STRIDE, off, n))
            out.append(torch.from_numpy(hb.reshape(-1)).cuda())
        return p, out, wires

    def run(label, kernels, fn, bufs, calls=CALLS, warm=4):
        for k in range(warm):
            seq.call("warm", kernels, lambda: fn(bufs[k % len(bufs)]))
        for k in range(calls):
            seq.call(label, kernels, lambda: fn(bufs[k % len(bufs)]))
        torch.cuda.synchronize()

    def sha_of(res):
        torch.cuda.synchronize()
        return hashlib.sha256(res.cpu().numpy().tobytes()).hexdigest()

    # ---- C2 (4 rotating batches): calibration read, classify, release path, match_streams
    p2, c2, w2 = batches(2, 4, lambda b: b * N)
    ctx = pa.RxContext(dev)
    ctx.set_conn_table(pa.gen_conn_table(p2))
    res = torch.empty(N * 16, dtype=torch.uint8, device="cuda")
    sink = torch.zeros(4096, dtype=torch.int32, device="cuda")
    run("calib", ["calib_stream_read_kernel"], lambda d: tn.calib_stream_read(ctx, d, d.numel(), sink, stream), c2[:1], calls=6)
    plan["workloads"]["calib"] = {"bytes_per_launch": N * STRIDE}
    if want("c2_n1048576"):
        run("c2_n1048576", ["rx_classify_kernel"], lambda d: ctx.classify(d, STRIDE, FRAME_OFF, N, res, stream), c2)
        ctx.classify(c2[0], STRIDE, FRAME_OFF, N, res, stream)
        seq.calls.append(["gate", ["rx_classify_kernel"]])
        plan["gates"]["c2_n1048576"] = sha_of(res) == golden(2, 0, N)
        plan["workloads"]["c2_n1048576"] = {"algorithmic_bytes_per_launch": int(sum(w2) / 4) + 16 * N,
                                            "workload": "C2: 1514-B IPv4/TCP frames, 1 flow, 4 rotating resident batches"}
    full0 = None
    if want("c2_release_path_n1048576") or args.uncached:
        ctx.classify(c2[0], STRIDE, FRAME_OFF, N, res, stream)
        seq.calls.append(["gate", ["rx_classify_kernel"]])
        torch.cuda.synchronize()
        full0 = res.cpu().numpy().view(pa.RESULT_DTYPE).copy()
    if want("c2_release_path_n1048576"):
        ctx.set_verify(False)
        run("c2_release_path_n1048576", ["rx_classify_kernel"],
            lambda d: ctx.classify(d, STRIDE, FRAME_OFF, N, res, stream), c2)
        ctx.classify(c2[0], STRIDE, FRAME_OFF, N, res, stream)
        seq.calls.append(["gate", ["rx_classify_kernel"]])
        torch.cuda.synchronize()
        F = pa.rx.F
        exp = full0.copy()
        exp["flags"] = (exp["flags"] & ~np.uint16(F.TCP_OK | F.RFC_TCP_OK)) | np.uint16(F.TCP_UNCHECKED)
        exp["tcp_fold"] = 0xFFFF
        plan["gates"]["c2_release_path_n1048576"] = bool(np.array_equal(res.cpu().numpy().view(pa.RESULT_DTYPE), exp))
        ctx.set_verify(True)
        plan["workloads"]["c2_release_path_n1048576"] = {
            "algorithmic_bytes_per_launch": N * (64 + 16),
            "workload": "C2 through pn_set_verify(ctx, 0): the 64-B header window read + the 16-B record per frame"}
    flt = np.zeros(8, pa.STREAM_FILTER_DTYPE)
    for k in range(7):
        flt[k] = (int.from_bytes(bytes([10, 9, k, 1]), "little"), 0, int.from_bytes((5000 + k).to_bytes(2, "big"), "little"), 0, 0)
    flt[7] = (0, 0, 0, int.from_bytes((1234).to_bytes(2, "big"), "little"), 0)
    ids = torch.empty(N, dtype=torch.int32, device="cuda")
    ids_ref = None
    if want("match_streams_c2_n1048576") or args.uncached:
        ctx.match_streams(c2[0], STRIDE, FRAME_OFF, N, flt, ids, stream)
        seq.calls.append(["gate", ["match_streams_mask_kernel"]])
        torch.cuda.synchronize()
        ids_ref = ids.cpu().numpy().copy()
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from streams_np import match_streams_np

        plan["gates"]["match_streams_c2_n1048576"] = bool(np.array_equal(
            ids_ref[:65536].view(np.uint32), match_streams_np(np.ascontiguousarray(c2[0][:65536 * STRIDE].cpu().numpy()
                                                                                   .reshape(65536, STRIDE)), FRAME_OFF, flt)))
    if want("match_streams_c2_n1048576"):
        run("match_streams_c2_n1048576", ["match_streams_mask_kernel"],
            lambda d: ctx.match_streams(d, STRIDE, FRAME_OFF, N, flt, ids, stream), c2)
        plan["workloads"]["match_streams_c2_n1048576"] = {
            "algorithmic_bytes_per_launch": N * (64 + 4),
            "workload": "pn_match_streams over C2 (8 filters): the 64-B header window read + the 4-B stream id"}
    if args.uncached:
        hip = ctypes.CDLL("libamdhip64.so")
        hip.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
        hip.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
        hip.hipFree.argtypes = [ctypes.c_void_p]
        ubufs = []
        for b in range(4):
            ptr = ctypes.c_void_p()
            rc = hip.hipExtMallocWithFlags(ctypes.byref(ptr), N * STRIDE, 0x3)  # hipDeviceMallocUncached
            assert rc == 0 and ptr.value, f"hipExtMallocWithFlags(uncached) failed: {rc}"
            assert hip.hipMemcpy(ptr.value, c2[b].data_ptr(), N * STRIDE, 3) == 0  # device to device
            ubufs.append(ptr.value)
        torch.cuda.synchronize()
        run("uncached_match_streams_c2", ["match_streams_mask_kernel"],
            lambda d: ctx.match_streams(d, STRIDE, FRAME_OFF, N, flt, ids, stream), ubufs)
        ctx.match_streams(ubufs[0], STRIDE, FRAME_OFF, N, flt, ids, stream)
        seq.calls.append(["gate", ["match_streams_mask_kernel"]])
        torch.cuda.synchronize()
        plan["gates"]["uncached_match_streams_c2"] = bool(np.array_equal(ids.cpu().numpy(), ids_ref))
        ctx.set_verify(False)
        run("uncached_c2_release_path", ["rx_classify_kernel"],
            lambda d: ctx.classify(d, STRIDE, FRAME_OFF, N, res, stream), ubufs)
        ctx.classify(ubufs[0], STRIDE, FRAME_OFF, N, res, stream)
        seq.calls.append(["gate", ["rx_classify_kernel"]])
        torch.cuda.synchronize()
        rel_u = res.cpu().numpy().view(pa.RESULT_DTYPE).copy()
        ctx.classify(c2[0], STRIDE, FRAME_OFF, N, res, stream)
        seq.calls.append(["gate", ["rx_classify_kernel"]])
        torch.cuda.synchronize()
        plan["gates"]["uncached_c2_release_path"] = bool(np.array_equal(res.cpu().numpy().view(pa.RESULT_DTYPE), rel_u))
        ctx.set_verify(True)
        run("uncached_c2_n1048576", ["rx_classify_kernel"],
            lambda d: ctx.classify(d, STRIDE, FRAME_OFF, N, res, stream), ubufs)
        ctx.classify(ubufs[0], STRIDE, FRAME_OFF, N, res, stream)
        seq.calls.append(["gate", ["rx_classify_kernel"]])
        plan["gates"]["uncached_c2_n1048576"] = sha_of(res) == golden(2, 0, N)
        for u in ubufs:
            hip.hipFree(u)
        for lab, algo in (("uncached_match_streams_c2", N * 68), ("uncached_c2_release_path", N * 80),
                          ("uncached_c2_n1048576", int(sum(w2) / 4) + 16 * N)):
            plan["workloads"][lab] = {"algorithmic_bytes_per_launch": algo,
                                      "workload": "the C2 batches copied into hipDeviceMallocUncached memory"}
    ctx.close()
    del c2
    torch.cuda.empty_cache()

    # ---- C3, C5 (2 rotating batches each, as bench.py's secondary legs)
    for cfg in (3, 5):
        label = f"c{cfg}_n1048576"
        if not want(label):
            continue
        p, bufs, w = batches(cfg, 2, lambda b: b * N)
        ctx = pa.RxContext(dev)
        ctx.set_conn_table(pa.gen_conn_table(p))
        run(label, ["rx_classify_kernel"], lambda d: ctx.classify(d, STRIDE, FRAME_OFF, N, res, stream), bufs)
        ctx.classify(bufs[0], STRIDE, FRAME_OFF, N, res, stream)
        seq.calls.append(["gate", ["rx_classify_kernel"]])
        plan["gates"][label] = sha_of(res) == golden(cfg, 0, N)
        plan["workloads"][label] = {"algorithmic_bytes_per_launch": int(sum(w) / 2) + 16 * N,
                                    "workload": f"C{cfg}, 2 rotating resident batches"}
        ctx.close()
        del bufs
        torch.cuda.empty_cache()

    # ---- C4: rank 0's shard (2 Mi frames), 4 resident copies (bench.py's c4_shard and each rank at N>1)
    if want("c4_n2097152"):
        n4 = 1 << 21
        h4 = np.empty((n4, STRIDE), dtype=np.uint8)
        p, bufs, w = batches(4, 1, lambda b: 0, n=n4, hbuf=h4)
        del h4
        bufs += [bufs[0].clone() for _ in range(3)]
        res4 = torch.empty(n4 * 16, dtype=torch.uint8, device="cuda")
        ctx = pa.RxContext(dev)
        ctx.set_conn_table(pa.gen_conn_table(p))
        run("c4_n2097152", ["rx_classify_kernel"], lambda d: ctx.classify(d, STRIDE, FRAME_OFF, n4, res4, stream), bufs)
        ctx.classify(bufs[0], STRIDE, FRAME_OFF, n4, res4, stream)
        seq.calls.append(["gate", ["rx_classify_kernel"]])
        plan["gates"]["c4_n2097152"] = sha_of(res4) == golden(4, 0, n4)
        plan["workloads"]["c4_n2097152"] = {"algorithmic_bytes_per_launch": int(w[0]) + 16 * n4, "frames": n4,
                                            "workload": "C4 shard 0 (global frames [0, 2 Mi)), 4 resident copies"}
        ctx.close()
        del bufs, res4
        torch.cuda.empty_cache()

    # ---- TX fill at the ring layout (frame_off 2) and efvitcp's SendBuf layout (14), 2 rotating batches
    from oracle import pyoracle as orc

    p2 = pa.rx.GenParams.for_config(2)
    for off in (2, 14):
        label = f"tx_c2_n1048576/frame_off_{off}"
        if not want(label):
            continue
        ctx = pa.RxContext(dev)
        bufs = []
        for b in range(2):
            pa.gen_frames(p2, N, STRIDE, off, first_index=b * N, threads=16, out=host)
            if b == 0:
                exp = host[:4096].copy()
            d = torch.from_numpy(host.reshape(-1)).cuda()
            v = d.view(N, STRIDE)
            v[:, off + 24:off + 26] = 0x5A
            v[:, off + 50:off + 52] = 0xA5
            bufs.append(d)
        run(label, ["tx_fill_kernel", "tx_patch_kernel"], lambda d: ctx.tx_fill(d, STRIDE, off, N, None, pa.PN_TX_TCP, stream),
            bufs, calls=8)
        torch.cuda.synchronize()
        got = bufs[0][:4096 * STRIDE].cpu().numpy().reshape(4096, STRIDE)
        exp[:, off + 24:off + 26] = 0x5A
        exp[:, off + 50:off + 52] = 0xA5
        orc.tx_fill_batch(exp, STRIDE, off, 4096, None, orc.TX_TCP)
        plan["gates"][label] = bool(np.array_equal(got, exp))
        plan["workloads"][label] = {"algorithmic_bytes_per_launch": 1504 * N,
                                    "workload": f"pn_tx_fill (PN_TX_TCP) over C2 frames at frame_off {off}, both checksums "
                                                "scrambled, 2 rotating batches"}
        ctx.close()
        del bufs
        torch.cuda.empty_cache()

    # ---- experiments: TX fill variants of the tuning library (same frames and rotation as the product's TX legs)
    TX_FAMS = {40: ["tx_fill_kernel", "tx_patch_kernel"], 50: ["tx_fill_kernel", "tx_patch_wt_kernel"],
               51: ["tx_fill_kernel", "tx_patch_wt_kernel"], 52: ["tx_fill_kernel", "tx_patch_kernel", "tx_l2_release_kernel"],
               32: ["tx_fill_kernel", "tx_patch_sector_kernel"], 41: ["tx_fill_kernel"],
               13: ["tx_fill_kernel"], 14: ["tx_patch_kernel"]}  # 13 / 14: one phase alone (timing only, no gate)
    tx_vs = [int(v) for v in filter(None, args.tx_variants.split(","))]
    for off in (2, 14) if tx_vs else ():
        ctx = pa.RxContext(dev)
        bufs = []
        for b in range(2):
            pa.gen_frames(p2, N, STRIDE, off, first_index=b * N, threads=16, out=host)
            d = torch.from_numpy(host.reshape(-1)).cuda()
            v = d.view(N, STRIDE)
            v[:, off + 24:off + 26] = 0x5A
            v[:, off + 50:off + 52] = 0xA5
            bufs.append(d)
        ref = bufs[0].clone()
        ctx.tx_fill(ref, STRIDE, off, N, None, pa.PN_TX_TCP, stream)
        seq.calls.append(["gate", ["tx_fill_kernel", "tx_patch_kernel"]])
        for var in tx_vs:
            label = f"x_tx_v{var}/frame_off_{off}"
            run(label, TX_FAMS[var], lambda d: tn.tx_fill_variant(ctx, d, STRIDE, off, N, None, var, stream), bufs, calls=8)
            plan["workloads"][label] = {"algorithmic_bytes_per_launch": 1504 * N,
                                        "workload": f"TX fill tuning variant {var} at frame_off {off} (experiment)"}
            if var in (13, 14):
                continue
            chk = bufs[0].clone()
            chk.view(N, STRIDE)[:, off + 24:off + 26] = 0x5A
            chk.view(N, STRIDE)[:, off + 50:off + 52] = 0xA5
            tn.tx_fill_variant(ctx, chk, STRIDE, off, N, None, var, stream)
            seq.calls.append(["gate", TX_FAMS[var]])
            torch.cuda.synchronize()
            plan["gates"][label] = bool(torch.equal(chk, ref))
            del chk
        ctx.close()
        del bufs, ref
        torch.cuda.empty_cache()

    plan["calls"] = seq.calls
    os.makedirs(args.out, exist_ok=True)
    with open(os.path.join(args.out, "plan.json"), "w") as f:
        json.dump(plan, f)
    log(json.dumps(plan["gates"]))
    if not all(plan["gates"].values()):
        log("ERROR: a correctness gate failed")
        sys.exit(1)


if __name__ == "__main__":
    t0 = time.time()
    main()
    log(f"done in {time.time() - t0:.1f}s")
