#!/usr/bin/env python3
"""Kernel time of the same C2 batch by where it sits in HBM: allocate K 2-GiB buffers in order
(torch's caching allocator, then hipMalloc directly), copy the same frames into each, time
pn_classify on each in interleaved rounds (HIP events).  Prints per buffer its device address
and median ms.  A measurement, not part of any product path."""
import ctypes as C
import json
import os
import statistics
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch

    import pollnet_amd as pa

    k = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    cfg = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    n, stride, off = 1 << 20, 2048, 2
    p = pa.rx.GenParams.for_config(cfg)
    s = pa.gen_frames(p, n, stride, off)
    ctx = pa.RxContext(0)
    ctx.set_conn_table(pa.gen_conn_table(p))
    src = torch.from_numpy(s.reshape(-1)).cuda()
    hip = C.CDLL("libamdhip64.so.7")
    bufs = []

    class Raw:  # a raw device allocation seen by torch (for copy_)
        def __init__(self, ptr, nbytes):
            self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 2}

    def hip_alloc():
        ptr = C.c_void_p()
        assert hip.hipMalloc(C.byref(ptr), C.c_size_t(n * stride)) == 0
        return ptr.value

    for i in range(k):  # allocation kind x fill method, interleaved in allocation order
        b = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
        b.copy_(src)
        bufs.append(("torch_alloc+torch_copy", b.data_ptr(), b))
        b2 = torch.empty(n * stride, dtype=torch.uint8, device="cuda")
        assert hip.hipMemcpy(C.c_void_p(b2.data_ptr()), C.c_void_p(src.data_ptr()), C.c_size_t(n * stride), 3) == 0
        bufs.append(("torch_alloc+hipMemcpy", b2.data_ptr(), b2))
        p3 = hip_alloc()
        assert hip.hipMemcpy(C.c_void_p(p3), C.c_void_p(src.data_ptr()), C.c_size_t(n * stride), 3) == 0
        bufs.append(("hipMalloc+hipMemcpy", p3, None))
        p4 = hip_alloc()
        t4 = torch.as_tensor(Raw(p4, n * stride), device="cuda")
        assert t4.data_ptr() == p4
        t4.copy_(src)
        bufs.append(("hipMalloc+torch_copy", p4, t4))
    torch.cuda.synchronize()
    res = torch.empty(n * 16, dtype=torch.uint8, device="cuda")
    ref = torch.empty_like(res)
    st = torch.cuda.current_stream()
    ctx.classify(src, stride, off, n, ref, st)
    times = [[] for _ in bufs]
    for _ in range(8):
        for i, (_, ptr, _) in enumerate(bufs):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            ctx.classify(ptr, stride, off, n, res, st)
            e0.record(st)
            for _ in range(5):
                ctx.classify(ptr, stride, off, n, res, st)
            e1.record(st)
            e1.synchronize()
            times[i].append(e0.elapsed_time(e1) / 5)
    torch.cuda.synchronize()
    assert torch.equal(res, ref)
    out = {"config": cfg, "buffers": [{"kind": kd, "addr_gib": round(ptr / 2**30, 3), "ms": round(statistics.median(t), 5)}
                                      for (kd, ptr, _), t in zip(bufs, times)]}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
