"""ctypes wrapper over oracle/liboracle.so (plain-C restatement) and oracle/_ref
(the reference's own TcpStream.h compiled from /root/reference).

TEST INFRASTRUCTURE ONLY — the checker and the timed CPU baseline ("port").
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_tcpstream.so")

RESULT_DTYPE = np.dtype(
    [("conn_id", "<u4"), ("seq", "<u4"), ("payload_off", "<u2"), ("payload_len", "<i2"), ("flags", "<u2"), ("tcp_fold", "<u2")]
)
ENTRY_DTYPE = np.dtype([("key", "<u8"), ("conn_id", "<u4"), ("_pad", "<u4")])

_lib = C.CDLL(ORACLE_SO)
_vp, _u32, _u64, _i32 = C.c_void_p, C.c_uint32, C.c_uint64, C.c_int


class _Csum(C.Structure):
    _fields_ = [("sum", _u32)]


class _Table(C.Structure):
    _fields_ = [("tbl", _vp), ("total", _u32), ("max_table_size", _u32), ("max_conn", _u32), ("max_tw", _u32),
                ("mask", _u64), ("size", _u32)]


def _sig(name, res, *args):
    f = getattr(_lib, name)
    f.restype, f.argtypes = res, list(args)
    return f


_fold = _sig("orc_csum_fold", C.c_uint16, _Csum)
_add16 = _sig("orc_csum_add16", None, C.POINTER(_Csum), C.c_uint16)
_add32 = _sig("orc_csum_add32", None, C.POINTER(_Csum), _u32)
_addb = _sig("orc_csum_add_bytes", None, C.POINTER(_Csum), _vp, _u32)
_key = _sig("orc_conn_hash_key", _u64, _u32, C.c_uint16)
_tinit = _sig("orc_table_init", _i32, C.POINTER(_Table), _u32, _u32)
_tfree = _sig("orc_table_free", None, C.POINTER(_Table))
_tfind = _sig("orc_table_find", _u32, C.POINTER(_Table), _u64)
_tadd = _sig("orc_table_add", _i32, C.POINTER(_Table), _u64, _u32)
_tdel = _sig("orc_table_del", _i32, C.POINTER(_Table), _u64)
_frame = _sig("orc_classify_frame", None, _vp, _u32, _vp, _u32, _u64, _u32, _vp)
_batch = _sig("orc_classify_batch", None, _vp, _u32, _u32, _u32, _vp, _u32, _u64, _u32, _vp, _i32)
_release = _sig("orc_release_batch", None, _vp, _u32, _u32, _u32, _vp, _u32, _u64, _u32, _vp, _i32)
_refsum = _sig("orc_refsum_batch", None, _vp, _u32, _u32, _u32, _vp, _u32, _u64, _u32, _vp, _i32)
_unverified = _sig("orc_classify_batch_unverified", None, _vp, _u32, _u32, _u32, _vp, _u32, _u64, _u32, _vp, _i32)
_tx_build = _sig("orc_tx_build_batch", _i32, _u64, _u32, _vp, _u32, _u32, _u32, _vp, _vp)
_tx_fill_frame = _sig("orc_tx_fill_frame", _i32, _vp, _u32, _i32, C.c_uint16, _u32)
_tx_fill_batch = _sig("orc_tx_fill_batch", None, _vp, _u32, _u32, _u32, _vp, _u32, _i32)
_tx_cas = _sig("orc_tx_copy_and_sum_batch", None, _vp, _vp, _u32, _u32, _u32, _i32)

TX_TCP, TX_UDP_EFVI, TX_UDP = 0, 1, 2
TX_KINDS = {0: "data", 1: "syn", 2: "resend", 3: "rst", 4: "tw_ack", 5: "udp"}


class Csum:
    """CSum (Core.h:89-138)."""

    def __init__(self, s=0):
        self.c = _Csum(s)

    def add16(self, v):
        _add16(C.byref(self.c), v)

    def add32(self, v):
        _add32(C.byref(self.c), v)

    def add_bytes(self, b: bytes, n=None):
        buf = C.create_string_buffer(bytes(b) + b"\0\0", len(b) + 2)
        _addb(C.byref(self.c), buf, len(b) if n is None else n)

    @property
    def sum(self):
        return self.c.sum

    def fold(self):
        return int(_fold(self.c))


def conn_hash_key(ip_be: int, port_be: int) -> int:
    return int(_key(ip_be, port_be))


class Table:
    """Ordered linear-probe conn table restated in C (Core.h:558-682)."""

    def __init__(self, max_conn, max_tw):
        self.t = _Table()
        assert _tinit(C.byref(self.t), max_conn, max_tw) == 0

    def __del__(self):
        _tfree(C.byref(self.t))

    def find(self, key):
        return int(_tfind(C.byref(self.t), key))

    def add(self, key, cid):
        return int(_tadd(C.byref(self.t), key, cid))

    def delete(self, key):
        return int(_tdel(C.byref(self.t), key))

    def set_conn_id(self, key, cid):
        e = self.find(key)
        arr = self.entries(copy=False)
        assert arr[e]["key"] == key
        arr[e]["conn_id"] = cid

    @property
    def mask(self):
        return int(self.t.mask)

    @property
    def size(self):
        return int(self.t.size)

    def entries(self, copy=True):
        buf = (C.c_uint8 * (self.t.total * 16)).from_address(self.t.tbl)
        a = np.frombuffer(buf, dtype=ENTRY_DTYPE)
        return a.copy() if copy else a


def classify_frame(eth: bytes, avail: int, entries: np.ndarray, mask: int, max_conn: int) -> np.void:
    buf = C.create_string_buffer(bytes(eth).ljust(avail, b"\0"), avail)
    out = np.zeros(1, RESULT_DTYPE)
    ent = np.ascontiguousarray(entries, dtype=ENTRY_DTYPE)
    _frame(buf, avail, ent.ctypes.data, len(ent), mask, max_conn, out.ctypes.data)
    return out[0]


def classify_batch(slots: np.ndarray, stride: int, frame_off: int, n: int, entries: np.ndarray, mask: int,
                   max_conn: int, threads: int = 1, release: bool = False, ref_only: bool = False,
                   unverified: bool = False) -> np.ndarray:
    """release: the minimal release-path record (timing); unverified: the exact record of
    pn_classify under pn_set_verify(ctx, 0) (orc_classify_batch_unverified)."""
    assert slots.dtype == np.uint8 and slots.flags.c_contiguous and slots.size >= n * stride
    ent = np.ascontiguousarray(entries, dtype=ENTRY_DTYPE)
    out = np.zeros(n, RESULT_DTYPE)
    fn = _unverified if unverified else (_release if release else (_refsum if ref_only else _batch))
    fn(slots.ctypes.data, stride, frame_off, n, ent.ctypes.data, len(ent), mask, max_conn, out.ctypes.data, threads)
    return out


_chain = _sig("orc_chain_links", None, _vp, _u32, _u32, _u32, _vp, _u32, _u32, _u32, _vp)
LINK_MAX_FRAMES, LINK_MAX_CONNS = 1024, 4096  # PN_LINK_MAX_FRAMES / PN_LINK_MAX_CONNS


def chain_links(slots: np.ndarray, stride: int, frame_off: int, n: int, recs: np.ndarray, max_conn: int,
                max_frames: int = LINK_MAX_FRAMES, max_conns: int = LINK_MAX_CONNS) -> np.ndarray:
    """orc_chain_links: the u16 chain link of each frame of a classified batch (pn_service_post_linked)."""
    assert slots.dtype == np.uint8 and slots.flags.c_contiguous and slots.size >= n * stride
    r = np.ascontiguousarray(recs[:n], dtype=RESULT_DTYPE)
    out = np.zeros(n, np.uint16)
    _chain(slots.ctypes.data, stride, frame_off, n, r.ctypes.data, max_conn, max_frames, max_conns, out.ctypes.data)
    return out


# ---------------- the reference itself: TcpStream.h (oracle/_ref) ----------------
_ref = None


def ref_available() -> bool:
    return os.path.exists(REF_SO)


def _ref_lib():
    global _ref
    if _ref is None:
        _ref = C.CDLL(REF_SO)
        _ref.ref_filter_packet.restype = _i32
        _ref.ref_filter_packet.argtypes = [_vp, _u32, C.c_char_p, C.c_uint16, C.c_char_p, C.c_uint16]
        _ref.ref_handle_packet.restype = _i32
        _ref.ref_handle_packet.argtypes = [_vp, _u32, C.POINTER(_u32), C.POINTER(_u32)]
    return _ref


def ref_filter_packet(eth: bytes) -> bool:
    b = C.create_string_buffer(bytes(eth), len(eth))
    return bool(_ref_lib().ref_filter_packet(b, len(eth), None, 0, None, 0))


def ref_handle_packet(eth: bytes):
    """(payload_off, payload_len) as TcpStream::handlePacket hands them over, or None."""
    b = C.create_string_buffer(bytes(eth), len(eth))
    off, ln = _u32(), _u32()
    ok = _ref_lib().ref_handle_packet(b, len(eth), C.byref(off), C.byref(ln))
    return (off.value, ln.value) if ok else None


# ---- TX checksum generation (pn_tx_oracle.c) ----
def tx_build_batch(seed: int, n: int, stride: int = 2048, frame_off: int = 14, mode: int = TX_TCP):
    """Frames a reference sender would put on the wire (incremental CSum path): (slots, lens, kinds)."""
    slots = np.zeros((n, stride), dtype=np.uint8)
    lens = np.zeros(n, dtype=np.uint16)
    kinds = np.zeros(n, dtype=np.uint8)
    rc = _tx_build(seed, n, slots.ctypes.data, stride, frame_off, mode, lens.ctypes.data, kinds.ctypes.data)
    assert rc == 0, "orc_tx_build_batch: bad layout"
    return slots, lens, kinds


def tx_fill_batch(slots: np.ndarray, stride: int, frame_off: int, n: int, lens=None, mode: int = TX_TCP, threads: int = 1):
    """pn_tx_fill's contract recomputed from the bytes, in place."""
    assert slots.flags.c_contiguous and slots.dtype == np.uint8
    lp = None if lens is None else np.ascontiguousarray(lens, dtype=np.uint16)
    _tx_fill_batch(slots.ctypes.data, stride, frame_off, n, None if lp is None else lp.ctypes.data, mode, threads)


def tx_copy_and_sum_batch(slots: np.ndarray, out: np.ndarray, stride: int, frame_off: int, n: int, threads: int = 1):
    _tx_cas(slots.ctypes.data, out.ctypes.data, stride, frame_off, n, threads)


# ---------------- the reference itself: efvitcp/Core.h's hot-path code (oracle/_ref/libref_core.so) ----------------
REF_CORE_SO = os.path.join(HERE, "_ref", "libref_core.so")
_rc = None


def ref_core():
    """ctypes handle of libref_core.so (oracle/ref_core.cc: Core.h's CSum, headers, connHashKey,
    conn-table member functions and Core::checksum compiled verbatim), or None if not built."""
    global _rc
    if _rc is None and os.path.exists(REF_CORE_SO):
        lib = C.CDLL(REF_CORE_SO)
        for name, res, args in (
            ("ref_csum_fold", C.c_uint16, [_u32]),
            ("ref_csum_words", C.c_uint16, [_vp, _u32]),
            ("ref_conn_hash_key", _u64, [_u32, C.c_uint16]),
            ("ref_header_fields", None, [_vp, _vp]),
            ("ref_checksum", _i32, [_vp]),
            ("ref_onpack_head", None, [_vp, _vp, _vp, _vp]),
            ("ref_checksum_folds", _i32, [_vp, _vp, _vp]),
            ("ref_tx_data_segment", None, [_vp, _vp, _u32, _vp, _u32]),
            ("ref_efvi_udp_datagram", None, [_vp, _u32]),
            ("ref_table_new", _vp, []),
            ("ref_table_free", None, [_vp]),
            ("ref_table_add", _i32, [_vp, _u64, _u32]),
            ("ref_table_del", _i32, [_vp, _u64]),
            ("ref_table_set_conn_id", _i32, [_vp, _u64, _u32]),
            ("ref_table_find", _u32, [_vp, _u64]),
            ("ref_table_entries", _u32, [_vp, _vp, _vp, _vp]),
            ("ref_table_debug_exits", _i32, [_vp]),
            ("ref_table_total_size", _u32, []),
            ("ref_bench_new", _vp, [_vp, _vp, _u32]),
            ("ref_bench_free", None, [_vp]),
            ("ref_bench_batch", _u64, [_vp, _vp, _u32, _u32, _u32, _i32, _vp]),
            ("ref_release_batch", _u64, [_vp, _vp, _u32, _u32, _u32, _i32]),
        ):
            f = getattr(lib, name)
            f.restype, f.argtypes = res, args
        _rc = lib
    return _rc


class RefCoreTable:
    """Core<Conf>'s conn table run by the reference's own member functions (MaxConnCnt =
    MaxTimeWaitConnCnt = 256), driven as TcpServer / enterTW drive it."""

    def __init__(self):
        self.lib = ref_core()
        self.h = self.lib.ref_table_new()

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.ref_table_free(self.h)
            self.h = None

    def add(self, key, cid):
        return int(self.lib.ref_table_add(self.h, key, cid))

    def delete(self, key):
        return int(self.lib.ref_table_del(self.h, key))

    def set_conn_id(self, key, cid):
        return int(self.lib.ref_table_set_conn_id(self.h, key, cid))

    def find(self, key):
        return int(self.lib.ref_table_find(self.h, key))

    def entries(self):
        n = int(self.lib.ref_table_total_size())
        keys = np.zeros(n, np.uint64)
        cids = np.zeros(n, np.uint32)
        mask = C.c_uint64()
        got = self.lib.ref_table_entries(self.h, keys.ctypes.data, cids.ctypes.data, C.byref(mask))
        assert got == n
        out = np.zeros(n, ENTRY_DTYPE)
        out["key"], out["conn_id"] = keys, cids
        return out, int(mask.value)

    @property
    def debug_exits(self):
        return int(self.lib.ref_table_debug_exits(self.h))


class RefBench:
    """The reference's own per-frame code (Core::checksum, connHashKey + findConnEntry, the
    TIME_WAIT test, TcpConn::onPack's head; oracle/ref_core.cc ref_bench_batch) over a slot ring,
    with a MaxConnCnt = 1024 table holding the given entries: bench.py's CPU baseline of kind
    "reference".  batch() returns (digest, frames verified)."""

    def __init__(self, entries: np.ndarray):
        self.lib = ref_core()
        ent = np.ascontiguousarray(entries, dtype=ENTRY_DTYPE)
        live = ent[ent["key"] != np.uint64(1 << 63)]
        keys = np.ascontiguousarray(live["key"])
        cids = np.ascontiguousarray(live["conn_id"])
        self.h = self.lib.ref_bench_new(keys.ctypes.data, cids.ctypes.data, len(live))

    def __del__(self):
        if getattr(self, "h", None):
            self.lib.ref_bench_free(self.h)
            self.h = None

    def batch(self, slots: np.ndarray, stride: int, frame_off: int, n: int, threads: int = 1):
        assert slots.dtype == np.uint8 and slots.flags.c_contiguous and slots.size >= n * stride
        valid = _u32(0)
        d = self.lib.ref_bench_batch(self.h, slots.ctypes.data, stride, frame_off, n, threads, C.byref(valid))
        return int(d), int(valid.value)

    def release(self, slots: np.ndarray, stride: int, frame_off: int, n: int, threads: int = 1) -> int:
        """The release build's per-frame work (ref_release_batch: no Core::checksum); its digest equals
        records_digest(records, release=True)."""
        assert slots.dtype == np.uint8 and slots.flags.c_contiguous and slots.size >= n * stride
        return int(self.lib.ref_release_batch(self.h, slots.ctypes.data, stride, frame_off, n, threads))


def records_digest(rec: np.ndarray, release: bool = False) -> int:
    """ref_bench_batch's digest (oracle/ref_core.cc ref_frame_digest) computed from pn_result
    records: (IP_OK and TCP_OK, HIT, TW, conn_id on hit, payload_off, payload_len, seq).
    release: ref_release_batch's (no checksum verified: the first term is 0)."""
    u = np.uint64
    fl = rec["flags"].astype(u)
    verified = np.zeros(len(rec), u) if release else ((fl & u(3)) == u(3)).astype(u)
    hit = (fl >> u(2)) & u(1)
    tw = (fl >> u(3)) & u(1)
    conn = np.where(hit == u(1), rec["conn_id"].astype(u), u(0xFFFFFFFF))
    x = verified | (hit << u(1)) | (tw << u(2)) | (conn << u(3))
    plen = rec["payload_len"].astype(np.int64).astype(np.uint32).astype(u)
    with np.errstate(over="ignore"):
        x ^= ((rec["payload_off"].astype(u) << u(32)) | plen) * u(0x9E3779B97F4A7C15)
        x ^= rec["seq"].astype(u) * u(0xC2B2AE3D27D4EB4F)
        d = (x * u(0xD6E8FEB86659FD93)) ^ (x >> u(29))
        return int(d.sum(dtype=u))
