"""Regenerate the committed golden fixtures (run in the build container).

  edge_frames.npz   hand-made edge frames (tests/golden/frames.py) in 2048-B slots,
                    the conn table they are classified against, the oracle's
                    expected pn_result records, and — where the reference itself
                    can be run (oracle/_ref: TcpStream.h compiled from
                    /root/reference) — its filterPacket/handlePacket verdicts.
  config_slices.npz per BASELINE config C2..C5: sha256 of the first 4096 generated
                    slots and of the conn table, and the oracle's records for them.
  full_digests.json sha256 of the oracle's records over the full BASELINE batch
                    (C2, C3, C5: 1,048,576 frames; C4 shard 0 of 8: 2,097,152),
                    and "c4_shards": each of C4's 8 index shards (2,097,152 frames
                    each, global frames [r*2Mi, (r+1)*2Mi)), so every rank of an
                    N<=8 bench run gates its own shard.
                    "c2_shards": C2's frames [1Mi, 4Mi) in 3 batches (the N=1 bench's
                    rotating batches 1-3).  `python make_golden.py shards` refreshes
                    only these two keys.

The oracle is pinned by known_answers.json, loopback_frames.npz and oracle/_ref
(tests/test_oracle.py); these fixtures then pin the product against it.
"""
import hashlib
import json
import os
import struct
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, HERE)

import pollnet_amd as pa  # noqa: E402  (generator + table builder only)
from frames import FRAME_OFF, STRIDE, make_frame, to_slots  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402

SLICE = 4096
FULL = {2: 1 << 20, 3: 1 << 20, 5: 1 << 20, 4: 1 << 21}


def edge_cases(table):
    """Returns (frames, after-bytes map, names)."""
    ents, mask = table.snapshot()
    live = [e for e in ents if e["key"] != pa.PN_EMPTY_KEY]
    tw = [e for e in live if e["conn_id"] >= table.max_conn_cnt]
    conn = [e for e in live if e["conn_id"] < table.max_conn_cnt]

    def flow_of(key):
        ip = (key >> 15) & 0xFFFFFFFF
        port = (key & 0x7FFF) | ((key >> 32) & 0x8000)
        return ".".join(str((ip >> s) & 255) for s in (24, 16, 8, 0)), port

    c_ip, c_port = flow_of(int(conn[5]["key"]))
    t_ip, t_port = flow_of(int(tw[0]["key"]))
    pay = bytes((i * 37 + 11) & 255 for i in range(1460))
    F, names, after = [], [], {}

    def add(name, fr, aft=None):
        if aft is not None:
            after[len(F)] = aft
        F.append(fr)
        names.append(name)

    add("c2_valid", make_frame(c_ip, c_port, payload=pay))
    add("payload_bitflip", bytearray(make_frame(c_ip, c_port, payload=pay)))
    F[-1][200] ^= 0x04
    F[-1] = bytes(F[-1])
    fr = bytearray(make_frame(c_ip, c_port, payload=pay)); fr[14 + 8] ^= 1
    add("ttl_flip_ip_bad", bytes(fr))
    fr = bytearray(make_frame(c_ip, c_port, payload=pay)); fr[14 + 20 + 16] ^= 0xFF
    add("tcp_csum_field_bad", bytes(fr))
    add("odd_len_zero_pad", make_frame(c_ip, c_port, payload=pay[:961]))
    add("odd_len_nonzero_pad", make_frame(c_ip, c_port, payload=pay[:961]), b"\xa5")
    add("odd_len_1_nonzero_pad", make_frame(c_ip, c_port, payload=pay[:1]), b"\x5a")
    add("tot_len_1800", make_frame(c_ip, c_port, payload=(pay * 2)[:1760]))
    add("tot_len_2032_slot_end", make_frame(c_ip, c_port, payload=(pay * 2)[:1992]))
    add("tot_len_2033_trunc", make_frame(c_ip, c_port, payload=(pay * 2)[:1993]))
    add("tot_len_65535_trunc", make_frame(c_ip, c_port, payload=pay[:100], tot_len=65535, fix_tcp=False))
    add("tot_len_0_trunc", make_frame(c_ip, c_port, payload=pay[:10], tot_len=0))
    add("tot_len_19_trunc", make_frame(c_ip, c_port, payload=pay[:10], tot_len=19))
    add("tot_len_20", make_frame(c_ip, c_port, payload=b"", tot_len=20))
    add("tot_len_21", make_frame(c_ip, c_port, payload=b"", tot_len=21))
    add("doff_15", make_frame(c_ip, c_port, doff=15, payload=pay[:300]))
    add("doff_8_ts", make_frame(c_ip, c_port, doff=8, payload=pay[:300]))
    add("doff_0", make_frame(c_ip, c_port, doff=0, payload=pay[:300]))
    add("doff_3", make_frame(c_ip, c_port, doff=3, payload=pay[:300]))
    add("doff_15_short_negative_len", make_frame(c_ip, c_port, doff=15, payload=b"", tot_len=50, fix_tcp=False))
    for ihl in (6, 7, 10, 15):
        add(f"ihl_{ihl}_nop", make_frame(c_ip, c_port, ihl=ihl, payload=pay[:500]))
    add("ihl_6_eol_zero_opts", make_frame(c_ip, c_port, ihl=6, ip_opts=b"\0\0\0\0", payload=pay[:501]))
    add("ihl_15_odd_nonzero_pad", make_frame(c_ip, c_port, ihl=15, payload=pay[:333]), b"\x77")
    add("ihl_4", make_frame(c_ip, c_port, ihl=4, payload=pay[:100]))
    add("ihl_0", make_frame(c_ip, c_port, ihl=0, payload=pay[:100]))
    add("ipv6_ethertype", make_frame(c_ip, c_port, ether_type=0x86DD, payload=pay[:100]))
    add("udp_proto", make_frame(c_ip, c_port, proto=17, payload=pay[:100]))
    add("ip_version_6", make_frame(c_ip, c_port, version=6, payload=pay[:100]))
    add("miss_flow", make_frame("10.9.9.9", 55555, payload=pay[:700]))
    add("miss_flow_syn", make_frame("10.9.9.9", 55556, flags=0x02, seq=0xFFFFFFFF, payload=b""))
    add("tw_hit_fin", make_frame(t_ip, t_port, flags=0x11, payload=pay[:10]))
    add("tw_hit_rst", make_frame(t_ip, t_port, flags=0x04, payload=b""))
    add("conn_syn_ack", make_frame(c_ip, c_port, flags=0x12, seq=0x7FFFFFFF, payload=b""))
    add("all_flags", make_frame(c_ip, c_port, flags=0xFF, payload=pay[:64]))
    add("seq_wrap_syn", make_frame(c_ip, c_port, flags=0x02, seq=0xFFFFFFFF, payload=pay[:64]))
    add("port_msb_clear", make_frame(c_ip, 1234, payload=pay[:64]))
    add("all_zero_frame", bytes(64))
    add("all_ff_frame", bytes([0xFF]) * 1514)
    add("min_64B", make_frame(c_ip, c_port, payload=pay[:10]))
    add("pad_after_even_ignored", make_frame(c_ip, c_port, payload=pay[:962]), b"\xff\xff")
    # every live key of the table, to walk every probe run (adversarial cluster included)
    for k, e in enumerate(live):
        ip, port = flow_of(int(e["key"]))
        add(f"key_{k}", make_frame(ip, port, payload=pay[: (k * 13) % 1400], seq=k))
        # a key just above it: walks the run then stops on a larger key or EmptyKey
        add(f"key_{k}_plus1", make_frame(ip, (port + 1) & 0xFFFF, payload=pay[:3], seq=k))
    return F, after, names


def digest(a: np.ndarray) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def records_digest(cfg, first, n, threads):
    """sha256 of the oracle's records over global frames [first, first+n) of config cfg,
    generated in 256K-frame chunks; also the wire bytes and the per-flag-bit counts."""
    p = pa.rx.GenParams.for_config(cfg)
    t = pa.gen_conn_table(p)
    e, m = t.snapshot()
    chunk = min(n, 1 << 18)
    h = hashlib.sha256()
    wire = 0
    flags_hist = np.zeros(16, np.int64)
    buf = np.empty((chunk, STRIDE), np.uint8)
    for lo in range(0, n, chunk):
        pa.gen_frames(p, chunk, STRIDE, FRAME_OFF, first_index=first + lo, threads=threads, out=buf)
        rr = orc.classify_batch(buf, STRIDE, FRAME_OFF, chunk, e, m, t.max_conn_cnt, threads=threads)
        h.update(rr.tobytes())
        wire += pa.wire_bytes(buf, STRIDE, FRAME_OFF, chunk)
        for bit in range(14):
            flags_hist[bit] += int(((rr["flags"] >> bit) & 1).sum())
    return {"n": n, "records_sha256": h.hexdigest(), "wire_bytes": wire, "flag_bit_counts": flags_hist[:14].tolist(),
            "seed": p.seed}


C4_SHARDS, C4_SHARD_N = 8, 1 << 21  # BASELINE configs[3]: 16 Mi frames over 8 GPUs


def c4_shards(threads):
    out = []
    for r in range(C4_SHARDS):
        d = records_digest(4, r * C4_SHARD_N, C4_SHARD_N, threads)
        d["first_index"] = r * C4_SHARD_N
        out.append(d)
        print(f"c4 shard {r}: {d['records_sha256'][:16]} wire={d['wire_bytes']}")
    return out


def c2_batches(threads):
    """C2 global frames [b*1Mi, (b+1)*1Mi), b = 1..3: the bench's N=1 rotating batches 1-3
    (batch 0 is the "c2" entry), so every timed batch is gated."""
    out = []
    for b in range(1, 4):
        d = records_digest(2, b << 20, 1 << 20, threads)
        d["first_index"] = b << 20
        out.append(d)
        print(f"c2 batch {b}: {d['records_sha256'][:16]}")
    return out


def main():
    threads = min(16, os.cpu_count() or 1)
    if sys.argv[1:] == ["shards"]:
        path = os.path.join(HERE, "full_digests.json")
        with open(path) as f:
            full = json.load(f)
        full["c4_shards"] = c4_shards(threads)
        full["c2_shards"] = c2_batches(threads)
        with open(path, "w") as f:
            json.dump(full, f, indent=1)
        return
    # ---- edge frames, classified against the C5 table (1024 conns, 32 TW, adversarial run) ----
    p5 = pa.rx.GenParams.for_config(5)
    table = pa.gen_conn_table(p5)
    ents, mask = table.snapshot()
    frames, after, names = edge_cases(table)
    slots = to_slots(frames, after=after)
    exp = orc.classify_batch(slots, STRIDE, FRAME_OFF, len(frames), ents, mask, table.max_conn_cnt)
    ref_filter = np.full(len(frames), -1, np.int8)
    ref_handle = np.full((len(frames), 2), -1, np.int64)
    if orc.ref_available():
        for i, f in enumerate(frames):
            eth = bytes(slots[i, FRAME_OFF:])  # the slot as the NIC left it
            ref_filter[i] = orc.ref_filter_packet(eth)
            h = orc.ref_handle_packet(eth)
            if h is not None:
                ref_handle[i] = h
    np.savez_compressed(os.path.join(HERE, "edge_frames.npz"), slots=slots, names=np.array(names), entries=ents,
                        mask=mask, max_conn=table.max_conn_cnt, expected=exp, ref_filter=ref_filter,
                        ref_handle=ref_handle, stride=STRIDE, frame_off=FRAME_OFF)
    print(f"edge_frames: {len(frames)} frames, ref available: {orc.ref_available()}")

    # ---- config slices + full digests ----
    slices, full = {}, {}
    for cfg in (2, 3, 4, 5):
        p = pa.rx.GenParams.for_config(cfg)
        t = pa.gen_conn_table(p)
        e, m = t.snapshot()
        s = pa.gen_frames(p, SLICE, STRIDE, FRAME_OFF, threads=threads)
        r = orc.classify_batch(s, STRIDE, FRAME_OFF, SLICE, e, m, t.max_conn_cnt, threads=threads)
        slices[f"c{cfg}_slots_sha256"] = digest(s)
        slices[f"c{cfg}_table_sha256"] = digest(e)
        slices[f"c{cfg}_mask"] = m
        slices[f"c{cfg}_expected"] = r
        # full-size digest, generated in 256K-frame chunks
        full[f"c{cfg}"] = records_digest(cfg, 0, FULL[cfg], threads)
        print(f"c{cfg}: {full[f'c{cfg}']}")
    full["c4_shards"] = c4_shards(threads)
    full["c2_shards"] = c2_batches(threads)
    np.savez_compressed(os.path.join(HERE, "config_slices.npz"), **slices)
    with open(os.path.join(HERE, "full_digests.json"), "w") as f:
        json.dump(full, f, indent=1)


if __name__ == "__main__":
    main()
