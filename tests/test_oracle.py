"""Pin the CPU oracle (oracle/pn_oracle.c) before trusting it (CPU only).

Pins: RFC 1071 known answers, the survey's probes of the real efvitcp Core
(known_answers.json), real Linux-generated frames (loopback_frames.npz), and
the reference's own TcpStream.h compiled from /root/reference (oracle/_ref).
"""
import json
import os
import struct

import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

from frames import FRAME_OFF, STRIDE, be_sum, csum


@pytest.fixture(scope="module")
def ka(golden_dir):
    with open(os.path.join(golden_dir, "known_answers.json")) as f:
        return json.load(f)


def test_rfc1071_example(ka):
    b = bytes.fromhex(ka["rfc1071_bytes_hex"])
    c = orc.Csum()
    c.add_bytes(b)
    assert c.sum == ka["rfc1071_csum_le_sum"]
    assert c.fold() == ka["rfc1071_csum_fold"]
    # byte-order independence (RFC 1071 §2B): LE fold == byte-swapped BE checksum
    be = (~ka["rfc1071_be_folded_sum"]) & 0xFFFF
    assert c.fold() == ((be >> 8) | ((be & 0xFF) << 8))


def test_ipv4_header_example(ka):
    c = orc.Csum()
    c.add_bytes(bytes.fromhex(ka["ipv4_header_hex"]))
    assert c.fold() == ka["ipv4_header_fold"]


def test_csum_add32_and_odd_read():
    # add(uint32) = hi + lo halves (Core.h:101-104); add(p, odd len) reads one byte past (Core.h:113-117)
    c = orc.Csum()
    c.add32(0x12345678)
    assert c.sum == 0x1234 + 0x5678
    a, b = orc.Csum(), orc.Csum()
    a.add_bytes(b"\x01\x02\x03\x00", 3)
    b.add_bytes(b"\x01\x02\x03\xff", 3)
    assert a.sum == 0x0201 + 0x0003 and b.sum == 0x0201 + 0xFF03


def test_conn_hash_key_probe(ka):
    ip_be = int.from_bytes(bytes([10, 0, 0, 2]), "little")
    port_be = int.from_bytes((40000).to_bytes(2, "big"), "little")
    want = ka["conn_hash_key_10.0.0.2_40000"]
    assert orc.conn_hash_key(ip_be, port_be) == want
    assert pa.conn_hash_key(ip_be, port_be) == want


def test_table_growth_probe(ka):
    exp = ka["table_1024_1024"]
    t = orc.Table(1024, 1024)
    assert t.t.max_table_size == exp["max_table_size"] and t.t.total == exp["total_table_size"]
    assert t.mask == exp["initial_mask"]
    rng = np.random.default_rng(1)
    keys = set()
    while len(keys) < 1024:
        keys.add(int(rng.integers(0, 1 << 47)))
    for i, k in enumerate(sorted(keys)):
        assert t.add(k, i) == 0
    assert t.mask == exp["mask_after_1024_inserts"]


def _random_history(seed, n_steps, cluster_frac):
    rng = np.random.default_rng(seed)
    ops, live = [], {}
    for _ in range(n_steps):
        op = rng.random()
        if (op < 0.55 and len(live) < 512) or not live:
            if rng.random() < cluster_frac:  # same low 12 bits -> one long sorted run, spills past tbl_mask
                k = (int(rng.integers(0, 1 << 20)) << 15) | 0x777
            else:
                k = int(rng.integers(0, 1 << 48))
            if k in live:
                continue
            cid = int(rng.integers(0, 512))
            ops.append(("add", k, cid))
            live[k] = cid
        elif op < 0.9:
            k = list(live)[int(rng.integers(0, len(live)))]
            ops.append(("del", k, 0))
            del live[k]
        else:
            k = list(live)[int(rng.integers(0, len(live)))]
            ops.append(("set", k, 300))
            live[k] = 300
    return ops, live


def _apply(t, op, k, c):
    if op == "add":
        r = t.add(k, c)
    elif op == "del":
        r = t.delete(k)
    else:
        r = t.set_conn_id(k, c)
    assert r in (None, 0)


def _canonical(live, max_conn=256, max_tw=256, mask=None):
    t = pa.ConnTable(max_conn, max_tw)
    for k in sorted(live):
        t.add(k, live[k])
    return t


def test_oracle_table_matches_product_table():
    """Two independent restatements of Core.h:558-682 (C oracle, C++ product) agree
    entry-for-entry through a random add/del/relabel history with spread keys."""
    ops, live = _random_history(11, 6000, 0.0)
    ot, pt = orc.Table(256, 256), pa.ConnTable(256, 256)
    for i, (op, k, c) in enumerate(ops):
        _apply(ot, op, k, c)
        _apply(pt, op, k, c)
        if i % 250 == 0 or i == len(ops) - 1:
            pe, pm = pt.snapshot()
            oe = ot.entries()
            assert pm == ot.mask and np.array_equal(pe["key"], oe["key"])
            occ = pe["key"] != pa.PN_EMPTY_KEY
            assert np.array_equal(pe["conn_id"][occ], oe["conn_id"][occ])
    assert pt.repairs == 0
    for k, cid in live.items():
        idx, hit, c = pt.find(k)
        assert hit and c == cid and ot.find(k) == idx


def test_reference_rehash_defect_and_product_repair():
    """Core::tryExpandConnTbl (Core.h:650-682) loses keys when a spill run past the
    old mask is rehashed after first-segment keys moved into the upper half (the
    reference's debug build exits there, Core.h:665-669).  The literal oracle shows
    it; the product detects the same condition and rebuilds canonically."""
    ops, live = _random_history(7, 400, 0.5)
    ot, pt = orc.Table(256, 256), pa.ConnTable(256, 256)
    for op, k, c in ops:
        _apply(ot, op, k, c)
        _apply(pt, op, k, c)
    oe = ot.entries()
    lost = [k for k in live if oe[ot.find(k)]["key"] != k]
    assert lost, "history no longer triggers the reference defect"
    assert pt.repairs >= 1
    for k, cid in live.items():
        idx, hit, c = pt.find(k)
        assert hit and c == cid


def test_reference_literal_table_equals_oracle_through_the_defect():
    """PN_TABLE_REFERENCE_LITERAL: the product table runs tryExpandConnTbl's rehash exactly
    (Core.h:650-682), so on the defect history it equals the literal oracle byte for byte at
    every step (mask, every key, every occupied conn_id) and strands the same keys."""
    ops, live = _random_history(7, 400, 0.5)
    ot, lt = orc.Table(256, 256), pa.ConnTable(256, 256, reference_literal=True)
    assert lt.reference_literal
    for op, k, c in ops:
        _apply(ot, op, k, c)
        _apply(lt, op, k, c)
        le, lm = lt.snapshot()
        oe = ot.entries()
        assert lm == ot.mask and np.array_equal(le["key"], oe["key"])
        occ = le["key"] != pa.PN_EMPTY_KEY
        assert np.array_equal(le["conn_id"][occ], oe["conn_id"][occ])
    assert lt.repairs == 0
    lost = [k for k in live if not lt.find(k)[1]]
    assert lost and lost == [k for k in live if oe[ot.find(k)]["key"] != k]


def test_product_table_is_canonical_under_clustered_history():
    """Ordered hashing has one layout per key set; the product keeps it through
    adds, backward-shift deletes, expansions and repairs (clustered keys)."""
    for seed in (3, 5, 7):
        ops, live = _random_history(seed, 5000, 0.5)
        pt = pa.ConnTable(256, 256)
        for op, k, c in ops:
            _apply(pt, op, k, c)
        pe, pm = pt.snapshot()
        ce, cm = _canonical(live).snapshot()
        if pm == cm:
            assert np.array_equal(pe["key"], ce["key"])
        for k, cid in live.items():
            _, hit, c = pt.find(k)
            assert hit and c == cid


def test_loopback_frames_real_kernel(golden_dir):
    d = np.load(os.path.join(golden_dir, "loopback_frames.npz"))
    slots, L = d["slots"], d["lengths"]
    ents = np.zeros(16, orc.ENTRY_DTYPE)
    ents["key"] = pa.PN_EMPTY_KEY
    res = orc.classify_batch(slots, int(d["stride"]), int(d["frame_off"]), len(L), ents, 15, 8)
    off = int(d["frame_off"])
    assert np.all(res["flags"] & pa.F.IP_OK), "Linux-built IPv4 headers must verify"
    for i in range(len(L)):
        eth = bytearray(slots[i, off:off + L[i]])
        ip = eth[14:]
        tot = struct.unpack("!H", ip[2:4])[0]
        doff = ip[32] >> 4
        assert res[i]["payload_off"] == 34 + 4 * doff
        assert res[i]["payload_len"] == tot - 20 - 4 * doff
        # CHECKSUM_PARTIAL: finish the sum the way Linux/NIC does (segment only, field as seed)...
        seg = bytes(ip[20:tot])
        fin = csum(seg)
        ip[20 + 16:20 + 18] = struct.pack("!H", fin)
        s2 = np.zeros((1, STRIDE), np.uint8)
        s2[0, FRAME_OFF:FRAME_OFF + L[i]] = np.frombuffer(bytes(eth[:14]) + bytes(ip), np.uint8)
        r2 = orc.classify_batch(s2, STRIDE, FRAME_OFF, 1, ents, 15, 8)
        # ...and the oracle's pseudo-header + segment sum must now verify (Core.h:459-466)
        assert r2[0]["flags"] & pa.F.TCP_OK and r2[0]["tcp_fold"] == 0


def test_edge_fixture_against_reference_tcpstream(golden_dir):
    """oracle/_ref = the reference's own TcpStream.h: filterPacket and the IHL=5 payload split."""
    d = np.load(os.path.join(golden_dir, "edge_frames.npz"))
    exp, rf, rh = d["expected"], d["ref_filter"], d["ref_handle"]
    assert (rf >= 0).all(), "fixture was made without oracle/_ref"
    slots, off = d["slots"], int(d["frame_off"])
    for i in range(len(exp)):
        ver = slots[i, off + 14] >> 4
        if ver == 4:  # filterPacket checks ether_type/protocol, efvitcp's NOT_TCP also the version
            assert bool(exp[i]["flags"] & pa.F.NOT_TCP) == (not rf[i]), d["names"][i]
        tot = int.from_bytes(bytes(slots[i, off + 16:off + 18]), "big")
        doff = slots[i, off + 14 + 32] >> 4
        if rh[i][0] >= 0:
            assert rh[i][0] == exp[i]["payload_off"], d["names"][i]
            if tot <= 1500:  # efvitcp clamps data_end at 1500 (TcpConn.h:472), TcpStream does not
                assert rh[i][1] == exp[i]["payload_len"], d["names"][i]
        else:  # TcpStream drops empty / negative payloads
            assert (tot - 20 - 4 * int(doff)) <= 0 or tot - 20 - 4 * int(doff) > (1 << 20) or int(exp[i]["payload_len"]) <= 0


def test_oracle_reproduces_committed_edge_fixture(golden_dir):
    d = np.load(os.path.join(golden_dir, "edge_frames.npz"))
    r = orc.classify_batch(d["slots"], int(d["stride"]), int(d["frame_off"]), len(d["expected"]), d["entries"],
                           int(d["mask"]), int(d["max_conn"]))
    assert np.array_equal(r, d["expected"])


def test_edge_fixture_semantics(golden_dir):
    """Spot-check named edge cases against hand-derived expectations."""
    d = np.load(os.path.join(golden_dir, "edge_frames.npz"))
    exp = {n: e for n, e in zip(d["names"], d["expected"])}
    F = pa.F
    assert exp["c2_valid"]["flags"] & (F.IP_OK | F.TCP_OK | F.HIT) == F.IP_OK | F.TCP_OK | F.HIT
    assert exp["c2_valid"]["payload_off"] == 54 and exp["c2_valid"]["payload_len"] == 1460
    assert not exp["payload_bitflip"]["flags"] & F.TCP_OK and exp["payload_bitflip"]["flags"] & F.IP_OK
    assert not exp["ttl_flip_ip_bad"]["flags"] & F.IP_OK and exp["ttl_flip_ip_bad"]["flags"] & F.TCP_OK
    assert exp["odd_len_zero_pad"]["flags"] & F.TCP_OK
    # reference reads the byte after an odd segment (Core.h:113-117): REF fails, RFC passes
    for n in ("odd_len_nonzero_pad", "odd_len_1_nonzero_pad"):
        assert not exp[n]["flags"] & F.TCP_OK and exp[n]["flags"] & F.RFC_TCP_OK, n
    assert exp["pad_after_even_ignored"]["flags"] & F.TCP_OK
    assert exp["tot_len_1800"]["payload_len"] == 1500 - 40
    assert exp["tot_len_2032_slot_end"]["flags"] & F.TCP_OK and not exp["tot_len_2032_slot_end"]["flags"] & F.TRUNC
    for n in ("tot_len_2033_trunc", "tot_len_65535_trunc", "tot_len_0_trunc", "tot_len_19_trunc"):
        assert exp[n]["flags"] & F.TRUNC and exp[n]["tcp_fold"] == 0xFFFF and not exp[n]["flags"] & F.TCP_OK, n
    assert exp["doff_0"]["payload_off"] == 34 and exp["doff_15"]["payload_off"] == 94
    assert exp["doff_15_short_negative_len"]["payload_len"] == 50 - 20 - 60
    for ihl in (6, 7, 10, 15):
        e = exp[f"ihl_{ihl}_nop"]
        assert e["flags"] & F.IHL_NE_5 and e["flags"] & F.RFC_IP_OK and e["flags"] & F.RFC_TCP_OK
        assert not e["flags"] & F.IP_OK  # REF sums 20 bytes only; NOP options break it
    assert exp["ihl_6_eol_zero_opts"]["flags"] & F.IP_OK  # zero options don't change the 20-B sum
    for n in ("ipv6_ethertype", "udp_proto", "ip_version_6"):
        assert exp[n]["flags"] & F.NOT_TCP, n
    assert exp["miss_flow"]["conn_id"] == pa.PN_MISS and not exp["miss_flow"]["flags"] & F.HIT
    assert exp["tw_hit_fin"]["flags"] & F.TW and exp["tw_hit_fin"]["conn_id"] >= int(d["max_conn"])
    assert exp["seq_wrap_syn"]["seq"] == 0  # 0xFFFFFFFF + syn
    assert exp["all_zero_frame"]["tcp_fold"] == 0xFFFF or exp["all_zero_frame"]["flags"] & F.TRUNC
    keys = [n for n in exp if n.startswith("key_") and not n.endswith("plus1")]
    assert all(exp[n]["flags"] & F.HIT for n in keys)


def test_config_slices_and_generator_determinism(golden_dir):
    import hashlib

    d = np.load(os.path.join(golden_dir, "config_slices.npz"))
    for cfg in (2, 3, 4, 5):
        p = pa.rx.GenParams.for_config(cfg)
        t = pa.gen_conn_table(p)
        e, m = t.snapshot()
        s = pa.gen_frames(p, 4096, STRIDE, FRAME_OFF, threads=4)
        assert hashlib.sha256(s.tobytes()).hexdigest() == str(d[f"c{cfg}_slots_sha256"])
        assert hashlib.sha256(e.tobytes()).hexdigest() == str(d[f"c{cfg}_table_sha256"])
        r = orc.classify_batch(s, STRIDE, FRAME_OFF, 4096, e, m, t.max_conn_cnt, threads=4)
        assert np.array_equal(r, d[f"c{cfg}_expected"])
        # shard determinism: generating [1000, 3000) directly equals the slice
        s2 = pa.gen_frames(p, 2000, STRIDE, FRAME_OFF, first_index=1000, threads=3)
        assert np.array_equal(s2, s[1000:3000])


def test_release_path_matches_full_path_fields():
    p = pa.rx.GenParams.for_config(3)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    s = pa.gen_frames(p, 2048)
    full = orc.classify_batch(s, STRIDE, FRAME_OFF, 2048, e, m, 1024)
    rel = orc.classify_batch(s, STRIDE, FRAME_OFF, 2048, e, m, 1024, release=True)
    for k in ("conn_id", "seq", "payload_off", "payload_len"):
        assert np.array_equal(full[k], rel[k])
    keep = pa.F.HIT | pa.F.TW | 0x1F0
    assert np.array_equal(full["flags"] & keep, rel["flags"])


@pytest.mark.parametrize("cfg", [3, 5])
def test_unverified_record_is_full_record_less_tcp_verdict(cfg):
    """orc_classify_batch_unverified (the expected record of pn_set_verify(ctx, 0)) computes no segment sum, yet equals
    the full record with the TCP verdict taken out (TCP_OK / RFC_TCP_OK cleared, TCP_UNCHECKED set, tcp_fold 0xFFFF):
    C3 / C5 frames (options, odd lengths, bad sums, TRUNC) and random bytes at every alignment class."""
    F = pa.F
    p = pa.rx.GenParams.for_config(cfg)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    s = pa.gen_frames(p, 4096)
    rng = np.random.default_rng(cfg)
    junk = rng.integers(0, 256, (512, STRIDE), dtype=np.uint8)
    junk[:, FRAME_OFF + 12:FRAME_OFF + 14] = (8, 0)
    junk[:, FRAME_OFF + 14] = 0x45
    junk[:, FRAME_OFF + 23] = 6
    s = np.ascontiguousarray(np.concatenate([s, junk]))
    n = len(s)
    full = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, 1024)
    got = orc.classify_batch(s, STRIDE, FRAME_OFF, n, e, m, 1024, unverified=True)
    exp = full.copy()
    exp["flags"] = (exp["flags"] & ~np.uint16(F.TCP_OK | F.RFC_TCP_OK)) | np.uint16(F.TCP_UNCHECKED)
    exp["tcp_fold"] = 0xFFFF
    assert np.array_equal(got, exp)
    assert (full["flags"] & F.TRUNC).any() or cfg == 3


# ---- chain links (orc_chain_links, the statement the GPU pass of pn_service_post_linked is checked against) ----

def _chain(perturb=(), n_flows=4, per_flow=6, verify=True, unknown=(), tw=(), max_conn=1024, **kw):
    import chainframes as cf
    import pollnet_amd as pa

    fr, flows = cf.build(n_flows, per_flow, perturb=perturb, unknown=unknown)
    s = cf.slots_of(fr)
    t = cf.table_for(pa, flows, max_conn=max_conn, tw=tw)
    e, m = t.snapshot()
    r = orc.classify_batch(s, STRIDE, FRAME_OFF, len(fr), e, m, t.max_conn_cnt, unverified=not verify)
    return orc.chain_links(s, STRIDE, FRAME_OFF, len(fr), r, t.max_conn_cnt, **kw).reshape(per_flow, n_flows).T


def test_chain_links_in_order_flows():
    """Interleaved in-order flows: every segment but a flow's first links back to the flow's previous frame."""
    got = _chain()
    assert (got[:, 0] == 0).all() and (got[:, 1:] == 4).all()
    single = _chain(n_flows=1, per_flow=40)  # one flow: each frame continues the one before it
    assert single[0, 0] == 0 and (single[0, 1:] == 1).all()


@pytest.mark.parametrize("kind", ["fin", "rst", "syn", "noack", "ack", "window", "dport", "pure_ack", "bad_ip"])
def test_chain_links_broken_at_a_frame(kind):
    """A frame TcpConn::onPack would not hand over as the next in-order segment with nothing else to do
    (TcpConn.h:650-725): it gets no link, and neither does its successor (whose predecessor it is)."""
    got = _chain(perturb=[(9, kind)])  # flow 1, segment 2
    exp = np.full((4, 6), 4, np.uint16)
    exp[:, 0] = 0
    exp[1, 2] = exp[1, 3] = 0
    assert np.array_equal(got, exp), (kind, got)


def test_chain_links_hole_and_retransmission():
    got = _chain(perturb=[(10, "hole")])  # flow 2, segment 2: 100 bytes past the next; the next frame is in order
    assert list(got[2]) == [0, 4, 0, 0, 4, 4]  # the hole's successor does not continue the hole's frame
    got = _chain(perturb=[(10, "retrans")])  # segment 2 repeats segment 1: its successor continues it again
    assert list(got[2]) == [0, 4, 0, 4, 4, 4]


def test_chain_links_tcp_verdict_by_path():
    """A bad TCP checksum breaks the chain where the checksum is verified, not on the release path (no verdict)."""
    assert list(_chain(perturb=[(9, "bad_tcp")])[1]) == [0, 4, 0, 0, 4, 4]
    assert list(_chain(perturb=[(9, "bad_tcp")], verify=False)[1]) == [0, 4, 4, 4, 4, 4]


def test_chain_links_skip_misses_and_time_wait():
    """Frames of unknown or TIME_WAIT flows are in no chain and break none."""
    got = _chain(unknown=(2,), tw=(3,))
    assert (got[2] == 0).all() and (got[3] == 0).all()
    assert (got[0, 1:] == 4).all() and (got[1, 1:] == 4).all()


def test_chain_links_bounds():
    """All 0 beyond the GPU pass's bounds: more frames than max_frames, or max_conn above max_conns."""
    assert (_chain(max_frames=23) == 0).all()
    assert (_chain(max_conn=8192) == 0).all()
    assert (_chain(max_conn=4096) != 0).any()
