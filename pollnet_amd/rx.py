"""ctypes bindings for libpollnet_amd.so (C-ABI: include/pollnet_amd.h).

Names follow the reference: ``conn_hash_key`` is ``connHashKey`` (efvitcp/Core.h:167-172),
``ConnTable.find/add/delete`` are ``findConnEntry/addConnEntry/delConnEntry``
(Core.h:558-605), ``RxContext.classify`` is the per-frame part of ``Core::pollNet``
(Core.h:494-552) plus ``TcpConn::onPack``'s payload split (TcpConn.h:469-473).
Errors surface as ``PollnetError`` carrying ``pn_last_error()`` (the reference's
``const char*`` / ``getLastError()`` convention, Core.h:253-383, Socket.h:47).
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass

import numpy as np

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpollnet_amd.so")

PN_EMPTY_KEY = 1 << 63
PN_MISS = 0xFFFFFFFF
PN_RECV_BUF_SIZE = 2048
PN_TX_TCP = 0       # efvitcp SendBuf::setOptDataLen / sumRst / resendUna (Core.h:157-163, 385-398; TcpConn.h:771-785)
PN_TX_UDP_EFVI = 1  # Efvi update_udp_pkt with the cached IPv4 sum (Efvi.h:405-411, 611-621), bit-exact
PN_TX_UDP = 2       # the same fields with CSum::fold (Core.h:94-98): always a verifying header checksum
PN_NOTIFY_MAX_FRAMES = 1024  # pn_classify_notify / pn_tx_fill_notify batch limit


class F:
    """pn_result.flags bits (include/pollnet_amd.h)."""

    IP_OK = 0x0001
    TCP_OK = 0x0002
    HIT = 0x0004
    TW = 0x0008
    FIN = 0x0010
    SYN = 0x0020
    RST = 0x0040
    PSH = 0x0080
    ACK = 0x0100
    IHL_NE_5 = 0x0200
    RFC_IP_OK = 0x0400
    RFC_TCP_OK = 0x0800
    NOT_TCP = 0x1000
    TRUNC = 0x2000
    BADOFF = 0x4000
    TCP_UNCHECKED = 0x8000  # pn_set_verify(ctx, 0): the release path, no TCP checksum


RESULT_DTYPE = np.dtype(
    [("conn_id", "<u4"), ("seq", "<u4"), ("payload_off", "<u2"), ("payload_len", "<i2"), ("flags", "<u2"), ("tcp_fold", "<u2")]
)
ENTRY_DTYPE = np.dtype([("key", "<u8"), ("conn_id", "<u4"), ("_pad", "<u4")])
# pn_stream_filter: TcpStream::initFilter's fields, network order, 0 = wildcard (TcpStream.h:32-37)
STREAM_FILTER_DTYPE = np.dtype([("src_ip", "<u4"), ("dst_ip", "<u4"), ("src_port", "<u2"), ("dst_port", "<u2"),
                                ("_pad", "<u4")])
PN_NO_STREAM = 0xFFFFFFFF
PN_MAX_STREAM_FILTERS = 64
assert RESULT_DTYPE.itemsize == 16 and ENTRY_DTYPE.itemsize == 16 and STREAM_FILTER_DTYPE.itemsize == 16


class PollnetError(RuntimeError):
    pass


def _load():
    # One HIP runtime per process: torch ships its own libamdhip64 with the same
    # SONAME (libamdhip64.so.7) as /opt/rocm's.  Loading torch first makes our
    # library bind to that already-loaded copy; the other order puts two HSA
    # runtimes in the process and the second one finds no device.
    try:
        import torch  # noqa: F401
    except ImportError:  # C++/ctypes users without torch get /opt/rocm's runtime
        pass
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} not built: run `make` (or __graft_entry__.build()); there is no CPU fallback for the RX path"
        )
    return ctypes.CDLL(LIB_PATH)


_lib = _load()
_c = ctypes
_vp, _u32, _u64, _i32, _u16 = _c.c_void_p, _c.c_uint32, _c.c_uint64, _c.c_int, _c.c_uint16


class _GenParams(_c.Structure):
    _fields_ = [("cfg", _u32), ("n_flows", _u32), ("n_tw_flows", _u32), ("max_conn_cnt", _u32), ("seed", _u64)]


def _sig(name, res, *args):
    fn = getattr(_lib, name)
    fn.restype = res
    fn.argtypes = list(args)
    return fn


_pn_conn_hash_key = _sig("pn_conn_hash_key", _u64, _u32, _u16)
_pn_table_create = _sig("pn_table_create", _i32, _u32, _u32, _c.POINTER(_vp))
_pn_table_create_ex = _sig("pn_table_create_ex", _i32, _u32, _u32, _u32, _c.POINTER(_vp))
_pn_table_flags = _sig("pn_table_flags", _u32, _vp)
_pn_table_destroy = _sig("pn_table_destroy", None, _vp)
_pn_table_find = _sig("pn_table_find", _i32, _vp, _u64, _c.POINTER(_u32), _c.POINTER(_i32), _c.POINTER(_u32))
_pn_table_add = _sig("pn_table_add", _i32, _vp, _u64, _u32)
_pn_table_del = _sig("pn_table_del", _i32, _vp, _u64)
_pn_table_set_conn_id = _sig("pn_table_set_conn_id", _i32, _vp, _u64, _u32)
_pn_table_entries = _sig("pn_table_entries", _vp, _vp, _c.POINTER(_u32), _c.POINTER(_u64))
_pn_table_max_conn_cnt = _sig("pn_table_max_conn_cnt", _u32, _vp)
_pn_table_size = _sig("pn_table_size", _u32, _vp)
_pn_table_repairs = _sig("pn_table_repairs", _u32, _vp)
_pn_open = _sig("pn_open", _i32, _i32, _c.POINTER(_vp))
_pn_close = _sig("pn_close", None, _vp)
_pn_last_error = _sig("pn_last_error", _c.c_char_p, _vp)
_pn_device_count = _sig("pn_device_count", _i32, _c.POINTER(_i32))
_pn_set_conn_table = _sig("pn_set_conn_table", _i32, _vp, _vp, _u32, _u64, _u32)
_pn_classify = _sig("pn_classify", _i32, _vp, _vp, _u32, _u32, _u32, _vp, _vp)
_pn_classify_indexed = _sig("pn_classify_indexed", _i32, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp)
_pn_tx_fill = _sig("pn_tx_fill", _i32, _vp, _vp, _u32, _u32, _u32, _vp, _u32, _vp)
_pn_classify_notify = _sig("pn_classify_notify", _i32, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _vp, _u32)
_pn_tx_fill_notify = _sig("pn_tx_fill_notify", _i32, _vp, _vp, _u32, _u32, _u32, _vp, _u32, _vp, _vp, _u32)
_pn_sync = _sig("pn_sync", _i32, _vp)
_pn_set_verify = _sig("pn_set_verify", _i32, _vp, _i32)
_pn_match_streams = _sig("pn_match_streams", _i32, _vp, _vp, _u32, _u32, _u32, _vp, _u32, _vp, _vp)
_pn_service_open = _sig("pn_service_open", _i32, _vp, _u32, _u32, _u32, _c.POINTER(_vp))
_pn_service_open_ex = _sig("pn_service_open_ex", _i32, _vp, _u32, _u32, _u32, _u32, _c.POINTER(_vp))
_pn_service_post = _sig("pn_service_post", _i32, _vp, _vp, _u32, _vp, _vp)
_pn_service_post_linked = _sig("pn_service_post_linked", _i32, _vp, _vp, _u32, _vp, _vp, _vp)
_pn_service_wait = _sig("pn_service_wait", _i32, _vp, _u32)
_pn_service_close = _sig("pn_service_close", _i32, _vp)
PN_SERVICE_WAVES = 64
PN_SERVICE_WAVES_PER_CU = 12
PN_SERVICE_MAX_WAVES = 4096
PN_LINK_MAX_FRAMES = 1024
PN_LINK_MAX_CONNS = 4096
PN_SERVICE_MAX_FRAMES = 1 << 20

# The seeded workload generator lives in its own library (include/pollnet_amd_gen.h), outside
# the product ABI; loaded on first use.
GEN_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpollnet_amd_gen.so")
_gen = {}


def _gen_fn(name, res, *args):
    if not _gen:
        if not os.path.exists(GEN_LIB_PATH):
            raise ImportError(f"{GEN_LIB_PATH} not built: run `make`")
        _gen["lib"] = ctypes.CDLL(GEN_LIB_PATH)
    fn = getattr(_gen["lib"], name)
    fn.restype = res
    fn.argtypes = list(args)
    return fn


def _check(rc, ctx=None, what=""):
    if rc != 0:
        msg = _pn_last_error(ctx).decode(errors="replace")
        raise PollnetError(f"{what} failed ({rc}): {msg}")


def conn_hash_key(ip_be: int, port_be: int) -> int:
    """connHashKey(ip, port) with network-byte-order inputs (Core.h:167-172)."""
    return int(_pn_conn_hash_key(ip_be & 0xFFFFFFFF, port_be & 0xFFFF))


def device_count() -> int:
    n = _i32(0)
    _pn_device_count(_c.byref(n))
    return n.value


PN_TABLE_REFERENCE_LITERAL = 1


class ConnTable:
    """Core's ordered linear-probe conn table (Core.h:178-182, 235-236, 558-682).
    reference_literal=True keeps tryExpandConnTbl's rehash exactly (Core.h:650-682), the
    key-stranding defect included; the default repairs it (``repairs`` counts)."""

    def __init__(self, max_conn_cnt: int, max_tw_cnt: int, reference_literal: bool = False):
        h = _vp()
        flags = PN_TABLE_REFERENCE_LITERAL if reference_literal else 0
        _check(_pn_table_create_ex(max_conn_cnt, max_tw_cnt, flags, _c.byref(h)), None, "pn_table_create_ex")
        self._h = h
        self.reference_literal = bool(_pn_table_flags(h) & PN_TABLE_REFERENCE_LITERAL)

    def __del__(self):
        if getattr(self, "_h", None):
            _pn_table_destroy(self._h)
            self._h = None

    @property
    def handle(self):
        return self._h

    def find(self, key: int):
        """findConnEntry: (entry_idx, hit, conn_id or PN_MISS)."""
        idx, hit, cid = _u32(), _i32(), _u32()
        _check(_pn_table_find(self._h, key, _c.byref(idx), _c.byref(hit), _c.byref(cid)), None, "pn_table_find")
        return idx.value, bool(hit.value), cid.value

    def add(self, key: int, conn_id: int):
        _check(_pn_table_add(self._h, key, conn_id), None, "pn_table_add")

    def delete(self, key: int):
        _check(_pn_table_del(self._h, key), None, "pn_table_del")

    def set_conn_id(self, key: int, conn_id: int):
        _check(_pn_table_set_conn_id(self._h, key, conn_id), None, "pn_table_set_conn_id")

    @property
    def max_conn_cnt(self) -> int:
        return int(_pn_table_max_conn_cnt(self._h))

    @property
    def size(self) -> int:
        return int(_pn_table_size(self._h))

    @property
    def repairs(self) -> int:
        return int(_pn_table_repairs(self._h))

    def snapshot(self):
        """(entries as an ENTRY_DTYPE numpy copy, tbl_mask)."""
        n, mask = _u32(), _u64()
        p = _pn_table_entries(self._h, _c.byref(n), _c.byref(mask))
        buf = (_c.c_uint8 * (n.value * 16)).from_address(p)
        return np.frombuffer(bytes(buf), dtype=ENTRY_DTYPE).copy(), int(mask.value)

    @property
    def mask(self) -> int:
        return self.snapshot()[1]


def _ptr(x):
    """Raw address of a torch tensor / numpy array / int."""
    if x is None:
        return None
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return x.data_ptr()
    if isinstance(x, np.ndarray):
        return x.ctypes.data
    raise TypeError(f"cannot take the address of {type(x)}")


def _hold(ctx, stream):
    """Keep a torch stream alive while the ctx may still use its handle (include/pollnet_amd.h:
    until the next pn_set_conn_table / pn_sync)."""
    h = _stream_handle(stream)
    if h is not None and not isinstance(stream, int) and h not in ctx._held:
        ctx._held[h] = stream
    return h


def _stream_handle(stream):
    if stream is None:
        return None
    if isinstance(stream, int):
        return stream
    return stream.cuda_stream  # torch.cuda.Stream


class RxContext:
    """A device context (pn_ctx): owns the device copy of the conn table."""

    def __init__(self, device: int = 0):
        h = _vp()
        _check(_pn_open(device, _c.byref(h)), None, "pn_open")
        self._h = h
        self.device = device
        self.max_conn_cnt = 0
        # handle -> stream object of the streams launched on since the last set / sync: the C-ABI
        # keeps those handles until then
        self._held = {}

    def close(self):
        if getattr(self, "_h", None):
            _pn_close(self._h)
            self._h = None

    __del__ = close

    def set_conn_table(self, table: ConnTable):
        entries, mask = table.snapshot()
        self.set_conn_entries(entries, mask, table.max_conn_cnt)

    def set_conn_entries(self, entries: np.ndarray, mask: int, max_conn_cnt: int):
        entries = np.ascontiguousarray(entries, dtype=ENTRY_DTYPE)
        _check(
            _pn_set_conn_table(self._h, entries.ctypes.data, len(entries), mask, max_conn_cnt), self._h, "pn_set_conn_table"
        )
        self.max_conn_cnt = max_conn_cnt
        self._held.clear()

    def set_verify(self, verify_tcp: bool):
        """pn_set_verify: False = the reference's release path (header lines only, no TCP checksum;
        records carry PN_F_TCP_UNCHECKED); True (default) = both checksums verified."""
        _check(_pn_set_verify(self._h, 1 if verify_tcp else 0), self._h, "pn_set_verify")

    def classify(self, frames_dev, slot_stride: int, frame_off: int, n: int, results_dev, stream=None):
        """Asynchronous launch on `stream` (torch.cuda.Stream, raw handle, or None = null stream)."""
        _check(
            _pn_classify(self._h, _ptr(frames_dev), slot_stride, frame_off, n, _ptr(results_dev), _hold(self, stream)),
            self._h,
            "pn_classify",
        )

    def classify_notify(self, frames, slot_stride: int, frame_off: int, n: int, results, done_word, token: int,
                        stream=None):
        """pn_classify_notify: as classify (n <= PN_NOTIFY_MAX_FRAMES), and the launch stores
        `token` to the u32 at done_word (pinned host memory) once every record is visible."""
        _check(_pn_classify_notify(self._h, _ptr(frames), slot_stride, frame_off, n, _ptr(results),
                                   _hold(self, stream), _ptr(done_word), token), self._h, "pn_classify_notify")

    def tx_fill_notify(self, frames, slot_stride: int, frame_off: int, n: int, done_word, token: int, lens=None,
                       mode: int = PN_TX_TCP, stream=None):
        """pn_tx_fill_notify: as tx_fill (n <= PN_NOTIFY_MAX_FRAMES) with the completion word."""
        _check(_pn_tx_fill_notify(self._h, _ptr(frames), slot_stride, frame_off, n, _ptr(lens), mode,
                                  _hold(self, stream), _ptr(done_word), token), self._h, "pn_tx_fill_notify")

    def classify_indexed(self, base, offsets, eth_mod16: int, n: int, avail: int, results, stream=None):
        """Frames at base + offsets[i] (u64; device or pinned host memory), all with
        offsets[i] % 16 == eth_mod16; asynchronous on `stream`."""
        _check(
            _pn_classify_indexed(self._h, _ptr(base), _ptr(offsets), eth_mod16, n, avail, _ptr(results),
                                 _hold(self, stream)),
            self._h,
            "pn_classify_indexed",
        )

    def tx_fill(self, frames_dev, slot_stride: int, frame_off: int, n: int, lens=None, mode: int = PN_TX_TCP,
                stream=None):
        """TX checksum fill in place (pn_tx_fill): IP + TCP checksums of n outgoing frames
        (mode PN_TX_TCP), or the IPv4 checksum of UDP frames (PN_TX_UDP_EFVI: Efvi's
        cached fold bit for bit; PN_TX_UDP: CSum::fold).  lens (device u16 per
        frame, optional) sets tot_len first, as setOptDataLen / update_udp_pkt do.
        Asynchronous on `stream`."""
        _check(_pn_tx_fill(self._h, _ptr(frames_dev), slot_stride, frame_off, n, _ptr(lens), mode,
                           _hold(self, stream)), self._h, "pn_tx_fill")

    def match_streams(self, frames, slot_stride: int, frame_off: int, n: int, filters: np.ndarray, stream_ids,
                      stream=None):
        """pn_match_streams: stream_ids[i] (u32, device or pinned memory) = the first filter
        (STREAM_FILTER_DTYPE, host array) frame i passes, PN_NO_STREAM if none."""
        flt = np.ascontiguousarray(filters, dtype=STREAM_FILTER_DTYPE)
        _check(_pn_match_streams(self._h, _ptr(frames), slot_stride, frame_off, n, flt.ctypes.data, len(flt),
                                 _ptr(stream_ids), _hold(self, stream)), self._h, "pn_match_streams")

    def sync(self):
        """pn_sync: every stream this ctx launched on has drained."""
        _check(_pn_sync(self._h), self._h, "pn_sync")
        self._held.clear()


@dataclass
class GenParams:
    cfg: int
    n_flows: int = 1024
    n_tw_flows: int = 0
    max_conn_cnt: int = 1024
    seed: int = 0

    @staticmethod
    def for_config(cfg: int) -> "GenParams":
        """C2 1 flow; C3 1024 flows / 32 TW; C4 1024 flows; C5 1024 flows / 32 TW."""
        seeds = {2: 0x5EED0002, 3: 0x5EED0003, 4: 0x5EED0004, 5: 0x5EED0005}
        if cfg == 2:
            return GenParams(2, 1, 0, 1024, seeds[2])
        if cfg == 4:
            return GenParams(4, 1024, 0, 1024, seeds[4])
        return GenParams(cfg, 1024, 32, 1024, seeds[cfg])

    def _c(self):
        return _GenParams(self.cfg, self.n_flows, self.n_tw_flows, self.max_conn_cnt, self.seed)


def gen_frames(params: GenParams, n: int, slot_stride: int = PN_RECV_BUF_SIZE, frame_off: int = 2, first_index: int = 0,
               threads: int = 0, out: np.ndarray | None = None) -> np.ndarray:
    """Deterministic synthetic ring slots (n, slot_stride) uint8 in host memory."""
    if out is None:
        out = np.empty((n, slot_stride), dtype=np.uint8)
    assert out.dtype == np.uint8 and out.flags.c_contiguous and out.size >= n * slot_stride
    threads = threads or min(16, os.cpu_count() or 1)
    p = params._c()
    gen = _gen_fn("pn_gen_frames", _i32, _c.POINTER(_GenParams), _u64, _u32, _vp, _u32, _u32, _i32)
    _check(gen(_c.byref(p), first_index, n, out.ctypes.data, slot_stride, frame_off, threads), None, "pn_gen_frames")
    return out


def gen_conn_table(params: GenParams, max_tw_cnt: int | None = None) -> ConnTable:
    t = ConnTable(params.max_conn_cnt, params.max_conn_cnt if max_tw_cnt is None else max_tw_cnt)
    p = params._c()
    _check(_gen_fn("pn_gen_conn_table", _i32, _c.POINTER(_GenParams), _vp)(_c.byref(p), t.handle), None,
           "pn_gen_conn_table")
    return t


def wire_bytes(slots: np.ndarray, slot_stride: int, frame_off: int, n: int) -> int:
    """Σ(14 + tot_len): the metric's numerator (wire frame bytes without FCS)."""
    return int(_gen_fn("pn_wire_bytes", _u64, _vp, _u32, _u32, _u32)(slots.ctypes.data, slot_stride, frame_off, n))


class RxService:
    """The resident classify service (pn_service_*): one launch, then batches posted through a mailbox in device memory
    (the large BAR; pinned host memory without one)
    and classified by the kernel already on the GPU.  Frames / results: pinned host or device memory.
    large_waves: a large post's wave count (pn_service_open_ex; 0 = the default, PN_SERVICE_WAVES_PER_CU per CU).
    Each post's frames and results objects are held until the post is waited for (or the service closed): the
    kernel reads and writes them until then."""

    def __init__(self, ctx: RxContext, slot_stride: int, frame_off: int, idle_ms: int = 200, large_waves: int = 0):
        h = _vp()
        _check(_pn_service_open_ex(ctx._h, slot_stride, frame_off, idle_ms, large_waves, _c.byref(h)), ctx._h,
               "pn_service_open")
        self._h, self._ctx = h, ctx
        self._inflight = {}  # post id -> (frames, results): alive until the post completes
        self._last = None  # the last post's id (ids wrap at 2^32: "the last" is not the largest)

    def post(self, frames, n: int, results, links=None) -> int:
        """Non-blocking; returns the post's id (posts complete in order).  links (n u16, pinned host or device
        memory): the post's chain links as well (pn_service_post_linked, n <= PN_LINK_MAX_FRAMES)."""
        pid = _u32(0)
        if links is None:
            rc = _pn_service_post(self._h, _ptr(frames), n, _ptr(results), _c.byref(pid))
        else:
            rc = _pn_service_post_linked(self._h, _ptr(frames), n, _ptr(results), _ptr(links), _c.byref(pid))
        _check(rc, self._ctx._h, "pn_service_post")
        self._inflight[pid.value] = (frames, results, links)
        self._last = pid.value
        return pid.value

    def wait(self, post_id: int = 0):
        """Until post post_id's records are visible (0: the last post)."""
        _check(_pn_service_wait(self._h, post_id), self._ctx._h, "pn_service_wait")
        # posts complete in order: every post up to the one waited for is done
        last = post_id or self._last
        if last is None:
            return
        for k in [k for k in self._inflight if ((last - k) & 0xFFFFFFFF) < 0x80000000]:
            del self._inflight[k]

    def classify(self, frames, n: int, results, links=None):
        self.post(frames, n, results, links)
        self.wait()

    def close(self):
        if getattr(self, "_h", None):
            h, self._h = self._h, None
            try:
                _check(_pn_service_close(h), self._ctx._h, "pn_service_close")
            finally:
                self._inflight.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:  # interpreter teardown
            pass
