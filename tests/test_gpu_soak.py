"""Optional GPU soak (PN_SOAK=<seeds> to run; skipped otherwise): random slot contents and generated C3/C5 frames
over many seeds, random layouts (frame_off, stride, n), through the full path and the release path
(pn_set_verify(ctx, 0)), every record against the oracle.  The suite's parity tests fix their seeds; this widens
them without slowing the suite."""
import os

import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

pytestmark = [pytest.mark.gpu,
              pytest.mark.skipif(not os.environ.get("PN_SOAK"), reason="soak: set PN_SOAK=<number of seeds>")]
F = pa.rx.F


def release(exp):
    r = exp.copy()
    r["flags"] = (r["flags"] & ~np.uint16(F.TCP_OK | F.RFC_TCP_OK)) | np.uint16(F.TCP_UNCHECKED)
    r["tcp_fold"] = 0xFFFF
    return r


def test_random_layout_soak():
    import torch

    assert torch.cuda.is_available()
    seeds = int(os.environ["PN_SOAK"])
    ctx = pa.RxContext(0)
    offs = [0, 2, 4, 6, 8, 10, 12, 14, 18, 34, 50, 98, 126]
    strides = [112, 128, 256, 1536, 2048, 4096, 9216]
    checked = 0
    for seed in range(seeds):
        rng = np.random.default_rng(0x50A4 + seed)
        cfg = int(rng.choice([3, 5]))
        stride = int(rng.choice(strides))
        off = int(rng.choice([o for o in offs if o + 96 <= stride]))
        n = int(rng.integers(1, 40000 if stride <= 2048 else 4000))
        p = pa.rx.GenParams.for_config(cfg)
        t = pa.gen_conn_table(p)
        e, m = t.snapshot()
        s = pa.gen_frames(p, n, stride, off)
        # a quarter of the slots overwritten with random bytes (garbage headers, any tot_len / IHL / doff)
        junk = rng.random(n) < 0.25
        s[junk] = rng.integers(0, 256, size=(int(junk.sum()), stride), dtype=np.uint8)
        exp = orc.classify_batch(s, stride, off, n, e, m, t.max_conn_cnt, threads=8)
        ctx.set_conn_table(t)
        frames = torch.from_numpy(np.ascontiguousarray(s).reshape(-1)).cuda()
        res = torch.full(((n + 7) * 16,), 0xAB, dtype=torch.uint8, device="cuda")
        for verify in (True, False):
            ctx.set_verify(verify)
            ctx.classify(frames, stride, off, n, res, torch.cuda.current_stream())
            torch.cuda.synchronize()
            out = res.cpu().numpy()
            assert (out[n * 16:] == 0xAB).all(), f"seed {seed}: wrote past n"
            got = out[: n * 16].view(pa.RESULT_DTYPE)
            want = exp if verify else release(exp)
            bad = np.nonzero(got != want)[0]
            assert len(bad) == 0, (f"seed {seed} cfg {cfg} stride {stride} off {off} n {n} verify {verify}: "
                                   f"{len(bad)} records differ, first #{bad[0]}: {got[bad[0]]} vs {want[bad[0]]}")
            checked += n
        ctx.set_verify(True)
    ctx.close()
    print(f"soak: {seeds} seeds, {checked} records checked")


def test_tx_fill_soak():
    """pn_tx_fill over random layouts and modes (TCP, Efvi UDP, canonical UDP), with and without lens, against the
    oracle's recomputation (itself pinned to the reference's copyAndSum / setOptDataLen / update_udp_pkt)."""
    import torch

    assert torch.cuda.is_available()
    seeds = int(os.environ["PN_SOAK"])
    ctx = pa.RxContext(0)
    offs = [0, 2, 4, 6, 8, 10, 12, 14, 18, 34, 50, 66, 98, 114, 126]
    strides = [112, 1024, 2048, 2064, 4096, 16384]
    checked = 0
    for seed in range(seeds):
        rng = np.random.default_rng(0x7A0 + seed)
        mode = int(rng.integers(0, 3))
        stride = int(rng.choice(strides))
        off = int(rng.choice([o for o in offs if o + 96 <= stride]))
        n = int(rng.integers(1, 80000 if stride <= 2064 else 3000))
        avail = stride - off
        slots = rng.integers(0, 256, (n, stride), dtype=np.uint8)
        tot = rng.integers(0, avail + 64, n)
        sane = rng.random(n) < 0.6
        tot[sane] = rng.integers(40, max(41, avail - 14 + 1), int(sane.sum()))
        slots[:, off + 16] = (tot >> 8) & 0xFF
        slots[:, off + 17] = tot & 0xFF
        lens = rng.integers(0, 65536, n).astype(np.uint16)
        lens[rng.random(n) < 0.7] %= max(1, avail - 40)
        use_lens = bool(rng.integers(0, 2))
        exp = slots.copy()
        orc.tx_fill_batch(exp, stride, off, n, lens if use_lens else None, mode, threads=8)
        d = torch.from_numpy(slots.reshape(-1)).cuda()
        ln = torch.from_numpy(lens.view(np.int16)).cuda() if use_lens else None
        ctx.tx_fill(d, stride, off, n, ln, mode)
        torch.cuda.synchronize()
        got = d.cpu().numpy().reshape(slots.shape)
        bad = np.nonzero((got != exp).any(1))[0]
        assert len(bad) == 0, f"seed {seed}: mode {mode} stride {stride} off {off} n {n} lens {use_lens}: {bad[:5]}"
        checked += n
    ctx.close()
    print(f"tx soak: {seeds} seeds, {checked} frames checked")


def test_match_streams_soak():
    """pn_match_streams over random layouts, random frames (TCP/UDP/other, random tuples) and random filter sets
    (0-64 filters, wildcards, many overlapping), against the numpy restatement of filterPacket."""
    import torch

    from streams_np import match_streams_np

    assert torch.cuda.is_available()
    seeds = int(os.environ["PN_SOAK"])
    ctx = pa.RxContext(0)
    checked = 0
    for seed in range(seeds):
        rng = np.random.default_rng(0x57A + seed)
        stride = int(rng.choice([112, 128, 1536, 2048, 4096, 65536]))
        off = int(rng.choice([o for o in (2, 4, 6, 8, 10, 12, 14, 16, 18, 34) if o + 96 <= stride]))
        n = int(rng.integers(1, 60000 if stride <= 4096 else 500))
        slots = rng.integers(0, 256, (n, stride), dtype=np.uint8)
        # a small pool of tuples so the filters hit: ethertype / protocol mostly IPv4 / TCP
        hosts = rng.integers(0, 1 << 32, 6, dtype=np.uint64).astype(np.uint32)
        ports = rng.integers(0, 1 << 16, 6).astype(np.uint16)
        eth = slots[:, off:]
        eth[:, 12] = 0x08
        eth[:, 13] = np.where(rng.random(n) < 0.9, 0x00, 0x06)
        eth[:, 23] = np.where(rng.random(n) < 0.9, 6, 17)
        for col, pool in ((26, hosts), (30, hosts)):
            v = pool[rng.integers(0, len(pool), n)]
            eth[:, col:col + 4] = v.astype("<u4").view(np.uint8).reshape(n, 4)
        for col in (34, 36):
            v = ports[rng.integers(0, len(ports), n)]
            eth[:, col:col + 2] = v.astype("<u2").view(np.uint8).reshape(n, 2)
        nf = int(rng.integers(0, 65))
        flt = np.zeros(nf, pa.STREAM_FILTER_DTYPE)
        for k in range(nf):
            flt[k] = (int(hosts[rng.integers(0, 6)]) if rng.random() < 0.6 else 0,
                      int(hosts[rng.integers(0, 6)]) if rng.random() < 0.6 else 0,
                      int(ports[rng.integers(0, 6)]) if rng.random() < 0.6 else 0,
                      int(ports[rng.integers(0, 6)]) if rng.random() < 0.6 else 0, 0)
        want = match_streams_np(slots, off, flt) if nf else np.full(n, 0xFFFFFFFF, np.uint32)
        d = torch.from_numpy(np.ascontiguousarray(slots).reshape(-1)).cuda()
        ids = torch.full((n + 5,), -1, dtype=torch.int32, device="cuda")
        ctx.match_streams(d, stride, off, n, flt, ids, torch.cuda.current_stream())
        torch.cuda.synchronize()
        got = ids.cpu().numpy().view(np.uint32)
        assert (got[n:] == 0xFFFFFFFF).all(), f"seed {seed}: wrote past n"
        bad = np.nonzero(got[:n] != want)[0]
        assert len(bad) == 0, f"seed {seed}: stride {stride} off {off} n {n} filters {nf}: {len(bad)} ids differ"
        checked += n
    ctx.close()
    print(f"match soak: {seeds} seeds, {checked} frames checked")
