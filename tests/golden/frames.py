"""Independent Python frame builder for hand-made edge cases (test-only).

Builds Ethernet/IPv4/TCP frames byte by byte with RFC 791/793 checksums computed
big-endian in pure Python — a formulation shared with neither the oracle
(LE u16 CSum) nor the HIP kernel (dword dot products).
"""
import struct

STRIDE = 2048
FRAME_OFF = 2


def ip4(s):
    return bytes(int(x) for x in s.split("."))


def be_sum(b: bytes, acc=0):
    if len(b) & 1:
        b = b + b"\0"
    for i in range(0, len(b), 2):
        acc += (b[i] << 8) | b[i + 1]
    return acc


def csum(b: bytes, acc=0):
    s = be_sum(b, acc)
    while s >> 16:
        s = (s & 0xFFFF) + (s >> 16)
    return (~s) & 0xFFFF


def make_frame(src="10.0.0.2", sport=40000, dst="10.0.0.1", dport=1234, seq=0, ack=0, flags=0x18, payload=b"",
               ihl=5, doff=5, ip_opts=None, tcp_opts=None, tot_len=None, ether_type=0x0800, version=4, proto=6,
               ttl=64, fix_ip=True, fix_tcp=True, window=0xFFFF):
    hl, th = 4 * ihl, 4 * doff
    ip_opts = ip_opts if ip_opts is not None else bytes([1] * max(0, hl - 20))
    tcp_opts = tcp_opts if tcp_opts is not None else bytes([1] * max(0, th - 20))
    seg = struct.pack("!HHIIBBHHH", sport, dport, seq & 0xFFFFFFFF, ack & 0xFFFFFFFF, (doff & 15) << 4, flags, window, 0, 0)
    seg += tcp_opts[: max(0, th - 20)] + payload
    real_len = max(hl, 20) + len(seg)
    tl = real_len if tot_len is None else tot_len
    iph = struct.pack("!BBHHHBBH4s4s", (version << 4) | (ihl & 15), 0, tl & 0xFFFF, 7, 0x4000, ttl, proto, 0, ip4(src), ip4(dst))
    iph += ip_opts[: max(0, hl - 20)]
    if fix_ip and hl >= 20:
        iph = iph[:10] + struct.pack("!H", csum(iph[:hl])) + iph[12:]
    if fix_tcp:
        pseudo = ip4(src) + ip4(dst) + struct.pack("!BBH", 0, 6, len(seg))
        c = csum(seg, be_sum(pseudo))
        seg = seg[:16] + struct.pack("!H", c) + seg[18:]
    eth = b"\x02\x00\x00\x00\x00\x01\x02\x00\x00\x00\x00\x02" + struct.pack("!H", ether_type)
    return eth + iph + seg


def to_slots(frames, stride=STRIDE, frame_off=FRAME_OFF, after=None):
    """Place frames in zeroed slots; `after` maps frame index -> bytes written right after the frame."""
    import numpy as np

    slots = np.zeros((len(frames), stride), np.uint8)
    for i, f in enumerate(frames):
        f = f[: stride - frame_off]
        slots[i, frame_off:frame_off + len(f)] = np.frombuffer(f, np.uint8)
        if after and i in after:
            b = after[i]
            e = frame_off + len(f)
            slots[i, e:e + len(b)] = np.frombuffer(b, np.uint8)
    return slots
