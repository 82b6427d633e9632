"""numpy restatement of TcpStream::filterPacket (TcpStream.h:39-52) over a batch of slots,
first matching filter wins (test-only; pn_match_streams' C++ test pins it to the
reference's own filterPacket)."""
import numpy as np


def match_streams_np(slots, frame_off, filters, no_stream=0xFFFFFFFF):
    eth = slots[:, frame_off:frame_off + 64]
    ether_type = eth[:, 12].astype(np.uint32) | (eth[:, 13].astype(np.uint32) << 8)  # as stored (LE load)
    proto = eth[:, 14 + 9]

    def u32(o):
        return np.ascontiguousarray(eth[:, o:o + 4]).view("<u4")[:, 0]

    def u16(o):
        return np.ascontiguousarray(eth[:, o:o + 2]).view("<u2")[:, 0]

    src_ip, dst_ip, src_port, dst_port = u32(26), u32(30), u16(34), u16(36)
    ids = np.full(len(slots), no_stream, np.uint32)
    ok = (ether_type == 0x0008) & (proto == 6)
    for k in range(len(filters) - 1, -1, -1):  # the first filter that passes wins
        q = filters[k]
        m = ok.copy()
        if q["src_ip"]:
            m &= src_ip == q["src_ip"]
        if q["dst_ip"]:
            m &= dst_ip == q["dst_ip"]
        if q["src_port"]:
            m &= src_port == q["src_port"]
        if q["dst_port"]:
            m &= dst_port == q["dst_port"]
        ids[m] = k
    return ids
