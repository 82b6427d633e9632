"""The oracle and the product's conn table pinned against the reference's OWN code.

oracle/_ref/libref_core.so is efvitcp/Core.h's hot-path code compiled verbatim from
/root/reference (oracle/ref_core.cc, oracle/ref.mk): CSum (Core.h:89-138), the
EtherHeader/IpHeader/TcpHeader bitfield layouts (:51-87), connHashKey (:167-172),
Core::checksum (:448-472, the EFVITCP_DEBUG check, its exit(1) recorded instead of
taken), the conn table's member functions findConnEntry / addConnEntry /
delConnEntry / tryExpandConnTbl (:558-605, 650-682), and TcpConn::onPack's payload
statements (TcpConn.h:469-473).  Every field of every RX record is therefore checked
against the reference itself, on the committed edge fixtures, the BASELINE config
slices, random inputs and table histories."""
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import pollnet_amd as pa  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402

ref = orc.ref_core()
pytestmark = pytest.mark.skipif(ref is None, reason="oracle/_ref/libref_core.so not built (needs /root/reference)")


def test_csum_fold_and_word_sums_match_reference():
    rng = np.random.default_rng(1)
    sums = [0, 1, 0xFFFF, 0x10000, 0x1FFFE, 0x1FFFF, 0xFFFEFFFF, 0xFFFFFFFF] + list(
        rng.integers(0, 1 << 32, 20000, dtype=np.uint64))
    for s in sums:
        assert orc._fold(orc._Csum(int(s))) == ref.ref_csum_fold(int(s)), hex(int(s))
    for n in (0, 1, 2, 10, 750):  # up to a 1500-B segment's words
        for _ in range(50):
            w = rng.integers(0, 1 << 16, n, dtype=np.uint16)
            c = orc._Csum(0)
            for x in w:
                orc._add16(orc.C.byref(c), int(x))
            assert orc._fold(c) == ref.ref_csum_words(w.ctypes.data, n)


def test_conn_hash_key_matches_reference():
    rng = np.random.default_rng(2)
    ips = [0, 0xFFFFFFFF, 0x0100000A, 0x0200000A] + list(rng.integers(0, 1 << 32, 20000, dtype=np.uint64))
    ports = [0, 0xFFFF, 0x0080, 0x8000, 0x409C] + list(rng.integers(0, 1 << 16, 20000, dtype=np.uint64))
    for ip, port in zip(ips, ports):
        k = ref.ref_conn_hash_key(int(ip), int(port))
        assert k == orc._key(int(ip), int(port)) == pa.conn_hash_key(int(ip), int(port))


def _frames():
    """(slots, stride, frame_off, n, entries, mask, max_conn) of every committed fixture."""
    d = np.load(os.path.join(ROOT, "tests", "golden", "edge_frames.npz"))
    out = [(d["slots"], int(d["stride"]), int(d["frame_off"]), len(d["slots"]), d["entries"], int(d["mask"]),
            int(d["max_conn"]))]
    for cfg in (2, 3, 5):
        p = pa.rx.GenParams.for_config(cfg)
        t = pa.gen_conn_table(p)
        e, m = t.snapshot()
        out.append((pa.gen_frames(p, 4096), 2048, 2, 4096, e, m, t.max_conn_cnt))
    return out


def test_header_fields_match_reference_bitfields():
    """IpHeader.header_len / TcpHeader.data_offset / flag bits as the reference's structs read
    them (Core.h:57-87) equal the oracle's record fields (IHL_NE_5, FIN..ACK, seq + syn)."""
    out = np.zeros(11, np.uint32)
    checked = 0
    for slots, stride, off, n, e, m, mc in _frames():
        rec = orc.classify_batch(np.ascontiguousarray(slots), stride, off, n, e, m, mc)
        for i in range(n):
            eth = slots[i, off:]
            ref.ref_header_fields(np.ascontiguousarray(eth).ctypes.data, out.ctypes.data)
            f = int(rec["flags"][i])
            assert bool(f & pa.F.IHL_NE_5) == (out[0] != 5)
            for bit, v in ((pa.F.FIN, out[5]), (pa.F.SYN, out[6]), (pa.F.RST, out[7]), (pa.F.PSH, out[8]),
                           (pa.F.ACK, out[9])):
                assert bool(f & bit) == bool(v)
            assert int(rec["seq"][i]) == (int(out[10]) + int(out[6])) & 0xFFFFFFFF  # TcpConn.h:473
            checked += 1
    assert checked > 14000


def test_checksum_verdicts_match_reference_core_checksum():
    """Core::checksum (Core.h:448-472) — the reference's own verification, run on every fixture
    frame whose summed bytes lie inside its slot — gives the oracle's REF-mode IP_OK / TCP_OK
    verdicts and the folded TCP sum (pn_result.tcp_fold, the value the debug build prints)
    bit for bit (IHL assumed 5, odd segments summed with the byte after them)."""
    import ctypes

    ipf, tcpf = ctypes.c_uint32(), ctypes.c_uint32()
    checked = bad = 0
    for slots, stride, off, n, e, m, mc in _frames():
        rec = orc.classify_batch(np.ascontiguousarray(slots), stride, off, n, e, m, mc)
        for i in range(n):
            eth = slots[i, off:]
            tot = (int(eth[16]) << 8) | int(eth[17])
            if tot < 20 or 14 + tot + (tot & 1) > stride - off:  # the reference would read outside the slot
                assert rec["flags"][i] & pa.F.TRUNC or tot < 20
                continue
            v = ref.ref_checksum_folds(np.ascontiguousarray(eth).ctypes.data, ctypes.byref(ipf), ctypes.byref(tcpf))
            f = int(rec["flags"][i])
            assert bool(v & 1) == bool(f & pa.F.IP_OK), i
            assert bool(v & 2) == bool(f & pa.F.TCP_OK), i
            assert int(rec["tcp_fold"][i]) == tcpf.value, i  # the folded TCP sum itself
            checked += 1
            bad += (v != 3)
    assert checked > 14000 and bad > 100  # both verdicts occur


def test_payload_extent_matches_reference_onpack():
    """payload_off / payload_len / seq of every record equal what TcpConn::onPack's own first
    statements compute (TcpConn.h:469-473: data = tcp + doff*4, data_end = ip +
    min(tot_len, 1500), seq = ntohl(seq_num) + syn), compiled from the reference."""
    import ctypes

    off_, len_, seq_ = ctypes.c_uint32(), ctypes.c_int32(), ctypes.c_uint32()
    checked = 0
    for slots, stride, off, n, e, m, mc in _frames():
        rec = orc.classify_batch(np.ascontiguousarray(slots), stride, off, n, e, m, mc)
        for i in range(n):
            eth = np.ascontiguousarray(slots[i, off:])
            ref.ref_onpack_head(eth.ctypes.data, ctypes.byref(off_), ctypes.byref(len_), ctypes.byref(seq_))
            assert int(rec["payload_off"][i]) == off_.value, i
            assert int(rec["payload_len"][i]) == len_.value, i  # signed: < 0 on malformed frames
            assert int(rec["seq"][i]) == seq_.value, i
            checked += 1
    assert checked > 14000


def _history(seed, n_steps, cluster_frac):
    from test_oracle import _random_history

    return _random_history(seed, n_steps, cluster_frac)


@pytest.mark.parametrize("seed,steps,cluster", [(11, 3000, 0.0), (3, 3000, 0.5), (7, 400, 0.5)])
def test_conn_table_matches_reference_member_functions(seed, steps, cluster):
    """The same add / delete / relabel history through the reference's own findConnEntry /
    addConnEntry / delConnEntry / tryExpandConnTbl, the C oracle and the product table in
    reference-literal mode: identical masks, keys and occupied conn_ids at every step.  Where
    the reference's rehash strands keys (seed 7), its own debug check fires (Core.h:665-669)
    and the product's default mode repairs the layout."""
    ops, live = _history(seed, steps, cluster)
    rt, ot = orc.RefCoreTable(), orc.Table(256, 256)
    lt, pt = pa.ConnTable(256, 256, reference_literal=True), pa.ConnTable(256, 256)
    for op, k, c in ops:
        if op == "add":
            ro = ot.add(k, c)
            if ro == -2:  # MaxConnCnt + MaxTimeWaitConnCnt entries: the reference's callers never add then
                live.pop(k, None)
                continue
            assert rt.add(k, c) == ro
            lt.add(k, c)
            pt.add(k, c)
        elif op == "del":
            r = rt.delete(k)
            assert r == ot.delete(k)
            if r == 0:
                lt.delete(k)
            pt.delete(k)
        else:
            r = rt.set_conn_id(k, c)
            if r == 0:
                ot.set_conn_id(k, c)
                lt.set_conn_id(k, c)
            pt.set_conn_id(k, c)
        re_, rm = rt.entries()
        le, lm = lt.snapshot()
        oe = ot.entries()
        assert rm == lm == ot.mask
        assert np.array_equal(re_["key"], le["key"]) and np.array_equal(re_["key"], oe["key"])
        occ = re_["key"] != pa.PN_EMPTY_KEY
        assert np.array_equal(re_["conn_id"][occ], le["conn_id"][occ])
        assert np.array_equal(re_["conn_id"][occ], oe["conn_id"][occ])
    stranded = [k for k in live if re_[rt.find(k)]["key"] != k]
    # the product repairs exactly the expansions in which the reference's own debug check fires
    assert (rt.debug_exits > 0) == (pt.repairs > 0)
    if stranded:
        assert rt.debug_exits > 0
    if seed == 7:
        assert stranded
    if cluster == 0.0:
        assert rt.debug_exits == 0
    for k, cid in live.items():  # the product's default table finds every live key
        _, hit, got = pt.find(k)
        assert hit and got == cid


@pytest.mark.parametrize("cfg", [2, 3, 4, 5])
def test_reference_batch_digest_equals_oracle_records(cfg):
    """ref_bench_batch (bench.py's "reference" CPU baseline: the reference's own per-frame code over
    a slot ring, threaded) does the same work as the oracle: its digest over (verified, hit, TW,
    conn_id, payload_off, payload_len, seq) equals the one computed from the oracle's records."""
    p = pa.rx.GenParams.for_config(cfg)
    n = 1 << 14
    slots = pa.gen_frames(p, n, threads=4)
    entries, mask = pa.gen_conn_table(p).snapshot()
    rec = orc.classify_batch(slots, 2048, 2, n, entries, mask, p.max_conn_cnt, threads=4)
    rb = orc.RefBench(entries)
    for threads in (1, 3):
        digest, n_valid = rb.batch(slots, 2048, 2, n, threads)
        assert digest == orc.records_digest(rec)
        assert n_valid == int(((rec["flags"] & 3) == 3).sum())
    # the release build's work (ref_release_batch, no Core::checksum) against the records of pn_set_verify(ctx, 0)
    unv = orc.classify_batch(slots, 2048, 2, n, entries, mask, p.max_conn_cnt, threads=4, unverified=True)
    for threads in (1, 3):
        assert rb.release(slots, 2048, 2, n, threads) == orc.records_digest(unv, release=True)


@pytest.mark.gpu
def test_gpu_records_digest_equals_reference_batch():
    """The GPU's records for C5 frames (options, odd lengths, bad checksums, probe cluster) against
    the reference's own code run on this host: equal digests."""
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    p = pa.rx.GenParams.for_config(5)
    n = 1 << 15
    slots = pa.gen_frames(p, n, threads=4)
    table = pa.gen_conn_table(p)
    entries, mask = table.snapshot()
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        frames = torch.from_numpy(np.ascontiguousarray(slots).reshape(-1)).cuda()
        res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        ctx.classify(frames, 2048, 2, n, res, torch.cuda.current_stream())
        torch.cuda.synchronize()
        rec = res.cpu().numpy().view(pa.RESULT_DTYPE)
    finally:
        ctx.close()
    digest, _ = orc.RefBench(entries).batch(slots, 2048, 2, n, 4)
    assert digest == orc.records_digest(rec)


@pytest.mark.parametrize("frame_off", [2, 10, 18])
def test_random_bytes_match_reference(frame_off):
    """Arbitrary bytes (random header fields, random IHL / data offset / flags, tot_len
    anywhere from 0 to past the slot, odd and even; half of them with checksums that verify):
    every record field the reference's own Core::checksum and onPack head compute equals the
    oracle's, wherever the reference's reads stay inside the slot (elsewhere the oracle flags
    TRUNC, as the GPU does)."""
    import ctypes

    rng = np.random.default_rng(0xF022 + frame_off)
    n, stride = 6000, 2048
    slots = rng.integers(0, 256, (n, stride), dtype=np.uint8)
    tot = rng.integers(0, stride - frame_off + 64, n)
    sane = rng.random(n) < 0.6
    tot[sane] = rng.integers(20, 1501, int(sane.sum()))
    eth = frame_off
    slots[:, eth + 16] = (tot >> 8) & 0xFF
    slots[:, eth + 17] = tot & 0xFF
    filled = slots.copy()  # half the frames with checksums that verify (the TX fill's recomputation)
    orc.tx_fill_batch(filled, stride, frame_off, n, None, orc.TX_TCP)
    pick = rng.random(n) < 0.5
    slots[pick] = filled[pick]
    ent = np.zeros(16, pa.ENTRY_DTYPE)
    ent["key"] = pa.PN_EMPTY_KEY
    rec = orc.classify_batch(slots, stride, frame_off, n, ent, 15, 1)
    ipf, tcpf = ctypes.c_uint32(), ctypes.c_uint32()
    off_, len_, seq_ = ctypes.c_uint32(), ctypes.c_int32(), ctypes.c_uint32()
    checked = ok_both = 0
    for i in range(n):
        e = np.ascontiguousarray(slots[i, frame_off:])
        t = int(tot[i])
        f = int(rec["flags"][i])
        ref.ref_onpack_head(e.ctypes.data, ctypes.byref(off_), ctypes.byref(len_), ctypes.byref(seq_))
        assert int(rec["payload_off"][i]) == off_.value and int(rec["payload_len"][i]) == len_.value, i
        assert int(rec["seq"][i]) == seq_.value, i
        if t < 20 or 14 + t + (t & 1) > stride - frame_off:
            assert f & pa.F.TRUNC or t < 20, i
            continue
        v = ref.ref_checksum_folds(e.ctypes.data, ctypes.byref(ipf), ctypes.byref(tcpf))
        assert bool(v & 1) == bool(f & pa.F.IP_OK), i
        assert bool(v & 2) == bool(f & pa.F.TCP_OK), i
        assert int(rec["tcp_fold"][i]) == tcpf.value, i
        checked += 1
        ok_both += (v == 3)
    assert checked > 3000 and ok_both > 500  # both verdicts occur
