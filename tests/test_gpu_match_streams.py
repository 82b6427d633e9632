"""pn_match_streams (TcpStream filter on the GPU) through the Python binding: C3/C5 batches
and random bytes, 1..64 overlapping wildcard filters, vs a numpy filterPacket."""
import numpy as np
import pytest

import pollnet_amd as pa

from streams_np import match_streams_np

pytestmark = pytest.mark.gpu


def _ip(s):
    return int.from_bytes(bytes(int(x) for x in s.split(".")), "little")


def _port(p):
    return int.from_bytes(p.to_bytes(2, "big"), "little")


def _filters(rng, slots, frame_off, k):
    """k filters: some copied from frames in the batch (with random wildcards), some random."""
    f = np.zeros(k, pa.STREAM_FILTER_DTYPE)
    for i in range(k):
        j = int(rng.integers(len(slots)))
        eth = slots[j, frame_off:]
        f[i]["src_ip"] = int.from_bytes(bytes(eth[26:30]), "little") if rng.random() < 0.7 else 0
        f[i]["dst_ip"] = int.from_bytes(bytes(eth[30:34]), "little") if rng.random() < 0.5 else 0
        f[i]["src_port"] = int.from_bytes(bytes(eth[34:36]), "little") if rng.random() < 0.7 else 0
        f[i]["dst_port"] = int.from_bytes(bytes(eth[36:38]), "little") if rng.random() < 0.5 else 0
        if rng.random() < 0.2:
            f[i]["src_ip"] = _ip(f"10.9.{i}.1")
    f[0] = (0, _ip("10.0.0.1"), 0, _port(1234), 0)  # dst-only filter: every TCP frame to the server
    return f


@pytest.mark.parametrize("cfg,frame_off", [(3, 2), (5, 10), (3, 24), (5, 16)])
def test_match_streams_vs_numpy(cfg, frame_off):
    import torch

    rng = np.random.default_rng(cfg * 100 + frame_off)
    n = 20000
    p = pa.rx.GenParams.for_config(cfg)
    slots = pa.gen_frames(p, n, 2048, frame_off)
    junk = rng.integers(0, 256, (n // 4, 2048), dtype=np.uint8)  # non-IPv4/non-TCP and garbage
    slots[rng.choice(n, n // 4, replace=False)] = junk
    ctx = pa.RxContext(0)
    dev = torch.from_numpy(slots.reshape(-1)).cuda()
    out = torch.full((n + 7,), 0xAB, dtype=torch.int32, device="cuda")
    for k in (1, 8, 64):
        flt = _filters(rng, slots, frame_off, k) if k > 1 else np.array([(0, _ip("10.0.0.1"), 0, 0, 0)],
                                                                        pa.STREAM_FILTER_DTYPE)
        ctx.match_streams(dev, 2048, frame_off, n, flt, out, torch.cuda.current_stream())
        torch.cuda.synchronize()
        got = out.cpu().numpy().view(np.uint32)
        assert (got[n:] == 0xAB).all(), "wrote past n"
        exp = match_streams_np(slots, frame_off, flt)
        assert np.array_equal(got[:n], exp), (k, int(np.count_nonzero(got[:n] != exp)))
        assert (exp != pa.PN_NO_STREAM).any() and (exp == pa.PN_NO_STREAM).any()
    ctx.close()
