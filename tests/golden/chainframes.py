"""Chain workloads for the chain links (pn_service_post_linked, oracle orc_chain_links; test-only).

Flows that each send in-order segments, interleaved in ring order as a NIC delivers several connections' frames,
with perturbations at chosen frames that each break the chain in one known way (FIN, RST, SYN, no ACK, another ack
number or window or destination port, a hole, a retransmission, a pure ACK, a bad checksum, an unknown flow).
Built byte by byte with tests/golden/frames.py (RFC 791/793 checksums computed independently of the oracle)."""
import numpy as np

from frames import FRAME_OFF, STRIDE, make_frame, to_slots

ACK, PSH, FIN, SYN, RST = 0x10, 0x08, 0x01, 0x02, 0x04


def flow_addr(f):
    return f"10.1.{f >> 8}.{f & 255}", 20000 + f


def build(n_flows, per_flow, seed=1, perturb=(), lens=None, unknown=()):
    """frames[i] of flow i % n_flows, its segment i // n_flows; perturb: (i, kind) pairs.  Returns (frames, flows)
    where flows[f] = (src ip, src port) for the conn table (conn_id f).  Frames of flows in `unknown` use addresses no
    table holds."""
    rng = np.random.default_rng(seed)
    n = n_flows * per_flow
    if lens is None:
        lens = rng.integers(1, 1461, size=n)
    kinds = dict(perturb)
    nxt = {f: int(rng.integers(0, 1 << 32)) for f in range(n_flows)}
    ackn = {f: int(rng.integers(0, 1 << 32)) for f in range(n_flows)}
    frames, prev_len = [], {}
    for i in range(n):
        f = i % n_flows
        src, sport = flow_addr(f)
        if f in unknown:
            src = "10.9.9.9"
        ln = int(lens[i])
        seq, ack, flags, win, dport, ln_eff = nxt[f], ackn[f], ACK | PSH, 0xFFFF, 1234, ln
        k = kinds.get(i)
        kw = {}
        if k == "fin":
            flags |= FIN
        elif k == "rst":
            flags |= RST
        elif k == "syn":
            flags = SYN | ACK
        elif k == "noack":
            flags = PSH
        elif k == "ack":
            ack = (ack + 1460) & 0xFFFFFFFF
        elif k == "window":
            win = 0x7000
        elif k == "dport":
            dport = 1235
        elif k == "hole":
            seq = (seq + 100) & 0xFFFFFFFF
        elif k == "retrans":
            seq = (seq - prev_len[f]) & 0xFFFFFFFF
            ln_eff = prev_len[f]
        elif k == "pure_ack":
            ln_eff = 0
        elif k == "bad_tcp":
            kw["fix_tcp"] = False
        elif k == "bad_ip":
            kw["fix_ip"] = False
        payload = bytes((j * 7 + i) & 255 for j in range(ln_eff))
        frames.append(make_frame(src=src, sport=sport, seq=seq, ack=ack, flags=flags, payload=payload, window=win,
                                 dport=dport, **kw))
        if k not in ("hole", "retrans"):  # the flow's next byte (a hole or a retransmission does not advance it)
            nxt[f] = (seq + ln_eff + (1 if k in ("fin", "syn") else 0)) & 0xFFFFFFFF
        prev_len[f] = ln_eff
    return frames, [flow_addr(f) for f in range(n_flows)]


def table_for(pa, flows, max_conn=1024, tw=()):
    """A conn table holding flows[f] as conn_id f (TIME_WAIT ids for the flows in `tw`)."""
    import struct

    t = pa.ConnTable(max_conn, max_conn)
    for f, (ip, port) in enumerate(flows):
        ip_be = struct.unpack("<I", bytes(int(x) for x in ip.split(".")))[0]
        port_be = struct.unpack("<H", struct.pack("!H", port))[0]
        t.add(int(pa.conn_hash_key(ip_be, port_be)), max_conn + f if f in tw else f)
    return t


def slots_of(frames):
    return to_slots(frames, STRIDE, FRAME_OFF)
