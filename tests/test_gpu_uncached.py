"""GPU: the classify (verified and release path) and pn_match_streams on a ring in uncached device memory
(hipExtMallocWithFlags(hipDeviceMallocUncached)), the round-5 experiment on the 128-B line floor (DESIGN §4,
scripts/pmc_workloads.py --uncached): the records and stream ids must equal the oracle's on that allocation too.
C3 and C5 frames (mixed lengths, options, odd lengths, bad sums, TIME_WAIT and miss flows)."""
import ctypes

import numpy as np
import pytest

import pollnet_amd as pa
from oracle import pyoracle as orc

from frames import FRAME_OFF, STRIDE

pytestmark = pytest.mark.gpu
F = pa.rx.F


@pytest.fixture(scope="module")
def hip():
    import torch

    assert torch.cuda.is_available(), "GPU tests need an MI355X"
    torch.cuda.init()
    lib = ctypes.CDLL("libamdhip64.so")
    lib.hipExtMallocWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_size_t, ctypes.c_uint]
    lib.hipMemcpy.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    lib.hipFree.argtypes = [ctypes.c_void_p]
    lib.hipDeviceSynchronize.argtypes = []
    return lib


def uncached_copy(hip, host: np.ndarray) -> int:
    ptr = ctypes.c_void_p()
    assert hip.hipExtMallocWithFlags(ctypes.byref(ptr), host.nbytes, 0x3) == 0 and ptr.value  # hipDeviceMallocUncached
    assert hip.hipMemcpy(ptr.value, host.ctypes.data, host.nbytes, 1) == 0  # host to device
    return ptr.value


@pytest.mark.parametrize("cfg", [3, 5])
def test_uncached_ring_equals_oracle(hip, cfg):
    import torch

    sys_path_streams()
    from streams_np import match_streams_np

    n = 1 << 16
    p = pa.rx.GenParams.for_config(cfg)
    slots = np.ascontiguousarray(pa.gen_frames(p, n, threads=8))
    table = pa.gen_conn_table(p)
    e, m = table.snapshot()
    full = orc.classify_batch(slots, STRIDE, FRAME_OFF, n, e, m, table.max_conn_cnt, threads=8)
    unv = orc.classify_batch(slots, STRIDE, FRAME_OFF, n, e, m, table.max_conn_cnt, threads=8, unverified=True)
    flt = np.zeros(3, pa.STREAM_FILTER_DTYPE)
    flt[0] = (slots[5, FRAME_OFF + 26:FRAME_OFF + 30].view("<u4")[0], 0, slots[5, FRAME_OFF + 34:FRAME_OFF + 36].view("<u2")[0],
              0, 0)  # frame 5's flow
    flt[1] = (0, 0, 0, 0, 0)  # wildcard: every TCP frame
    flt[2] = flt[0]
    ids_exp = match_streams_np(slots, FRAME_OFF, flt)
    dev = uncached_copy(hip, slots)
    ctx = pa.RxContext(0)
    try:
        ctx.set_conn_table(table)
        res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
        s = torch.cuda.current_stream()
        ctx.classify(dev, STRIDE, FRAME_OFF, n, res, s)
        torch.cuda.synchronize()
        assert np.array_equal(res.cpu().numpy().view(pa.RESULT_DTYPE), full)
        ctx.set_verify(False)
        ctx.classify(dev, STRIDE, FRAME_OFF, n, res, s)
        torch.cuda.synchronize()
        assert np.array_equal(res.cpu().numpy().view(pa.RESULT_DTYPE), unv)
        ids = torch.empty(n, dtype=torch.int32, device="cuda")
        ctx.match_streams(dev, STRIDE, FRAME_OFF, n, flt, ids, s)
        torch.cuda.synchronize()
        assert np.array_equal(ids.cpu().numpy().view(np.uint32), ids_exp)
    finally:
        ctx.close()
        hip.hipFree(dev)


def sys_path_streams():
    import os
    import sys

    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
