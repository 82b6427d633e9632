"""ctypes bindings for libpollnet_amd_tuning.so (include/pollnet_amd_tuning.h).

Measurement only — never imported by the product path: the same-run bandwidth ceilings
that bench.py reports beside the production kernel, and (library built with
``make``, unless ``TUNING=0``) the A/B kernel variants the scripts under scripts/ time.  Every call
takes an open ``RxContext`` (pn_open)."""
from __future__ import annotations

import ctypes
import os

from . import rx

LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libpollnet_amd_tuning.so")
_c = ctypes
_vp, _u32, _u64, _i32 = _c.c_void_p, _c.c_uint32, _c.c_uint64, _c.c_int

if not os.path.exists(LIB_PATH):
    raise ImportError(f"{LIB_PATH} not built: run `make`")
_lib = ctypes.CDLL(LIB_PATH)


def _sig(name, res, *args):
    fn = getattr(_lib, name, None)
    if fn is None:  # the A/B variants exist only in a TUNING=1 build
        return None
    fn.restype = res
    fn.argtypes = list(args)
    return fn


_calib = _sig("pn_calib_stream_read", _i32, _vp, _vp, _u64, _vp, _vp)
_calib_slot = _sig("pn_calib_slot_read", _i32, _vp, _vp, _u32, _u32, _u32, _i32, _vp, _vp)
_calib_slot_var = _sig("pn_calib_slot_read_var", _i32, _vp, _vp, _u32, _u32, _vp, _i32, _vp, _vp)
_calib_rx_abl = _sig("pn_calib_classify_ablated", _i32, _vp, _vp, _u32, _u32, _u32, _vp, _vp)
_calib_tx_abl = _sig("pn_calib_tx_ablated", _i32, _vp, _vp, _u32, _u32, _u32, _vp)
_match_variant = _sig("pn_match_streams_variant", _i32, _vp, _vp, _u32, _u32, _u32, _vp, _u32, _vp, _vp, _i32)
_spin = _sig("pn_test_spin_wait", _i32, _vp, _vp, _u32, _vp)
_variant = _sig("pn_classify_variant", _i32, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _i32)
_idx_variant = _sig("pn_classify_indexed_variant", _i32, _vp, _vp, _vp, _u32, _u32, _u32, _vp, _vp, _i32)
_tx_variant = _sig("pn_tx_fill_variant", _i32, _vp, _vp, _u32, _u32, _u32, _vp, _i32, _vp)


def _need(fn, name):
    if fn is None:
        raise rx.PollnetError(f"{name} needs the tuning library built with its variants (`make`, not `make TUNING=0`)")
    return fn


def calib_stream_read(ctx, src_dev, nbytes: int, sink_dev, stream=None):
    """Front-to-back streaming read of `nbytes` (the chip's achievable read rate)."""
    rx._check(_calib(ctx._h, rx._ptr(src_dev), nbytes, rx._ptr(sink_dev), rx._stream_handle(stream)), ctx._h,
              "pn_calib_stream_read")


def calib_slot_read(ctx, src_dev, n_slots, stride, nbytes, sink_dev, stream=None, store_bytes=0):
    """The RX kernel's load pattern over the first `nbytes` of each slot, no arithmetic."""
    rx._check(_calib_slot(ctx._h, rx._ptr(src_dev), n_slots, stride, nbytes, store_bytes, rx._ptr(sink_dev),
                          rx._stream_handle(stream)), ctx._h, "pn_calib_slot_read")


def calib_slot_read_var(ctx, src_dev, n_slots, stride, lens_dev, sink_dev, stream=None, store_bytes=0):
    """The same over each frame's own lines (lens_dev: u32 per slot)."""
    rx._check(_calib_slot_var(ctx._h, rx._ptr(src_dev), n_slots, stride, rx._ptr(lens_dev), store_bytes,
                              rx._ptr(sink_dev), rx._stream_handle(stream)), ctx._h, "pn_calib_slot_read_var")


def calib_classify_ablated(ctx, frames_dev, slot_stride, frame_off, n, results_dev, stream=None):
    """The production RX kernel with the probe and lane reduction ablated (timing-only ceiling)."""
    rx._check(_calib_rx_abl(ctx._h, rx._ptr(frames_dev), slot_stride, frame_off, n, rx._ptr(results_dev),
                            rx._stream_handle(stream)), ctx._h, "pn_calib_classify_ablated")


def calib_tx_ablated(ctx, frames_dev, slot_stride, frame_off, n, stream=None):
    """The production two-launch TX fill with its lane reduction ablated (timing-only ceiling)."""
    rx._check(_calib_tx_abl(ctx._h, rx._ptr(frames_dev), slot_stride, frame_off, n, rx._stream_handle(stream)), ctx._h,
              "pn_calib_tx_ablated")


def match_streams_variant(ctx, frames, slot_stride, frame_off, n, filters, stream_ids, variant, stream=None):
    """pn_match_streams' kernel in form `variant` (1 cooperative, 0 per lane)."""
    import numpy as np

    flt = np.ascontiguousarray(filters, dtype=rx.STREAM_FILTER_DTYPE)
    rx._check(_match_variant(ctx._h, rx._ptr(frames), slot_stride, frame_off, n, flt.ctypes.data, len(flt),
                             rx._ptr(stream_ids), rx._stream_handle(stream), variant), ctx._h, "pn_match_streams_variant")


def spin_wait(go_host, done_host, max_ms: int, stream=None):
    """Test helper: hold `stream` until go_host[0] != 0 (pinned u32) or max_ms pass; then
    done_host[0] = 1 (released) or 2 (timed out).  Uses no ctx."""
    rx._check(_spin(rx._ptr(go_host), rx._ptr(done_host), max_ms, rx._stream_handle(stream)), None,
              "pn_test_spin_wait")


def classify_variant(ctx, frames_dev, slot_stride, frame_off, n, results_dev, stream, variant):
    rx._check(_need(_variant, "pn_classify_variant")(ctx._h, rx._ptr(frames_dev), slot_stride, frame_off, n,
                                                     rx._ptr(results_dev), rx._stream_handle(stream), variant),
              ctx._h, "pn_classify_variant")


def classify_indexed_variant(ctx, base, offsets, eth_mod16, n, avail, results, stream, variant):
    rx._check(_need(_idx_variant, "pn_classify_indexed_variant")(ctx._h, rx._ptr(base), rx._ptr(offsets), eth_mod16, n,
                                                                 avail, rx._ptr(results), rx._stream_handle(stream),
                                                                 variant), ctx._h, "pn_classify_indexed_variant")


def tx_fill_variant(ctx, frames_dev, slot_stride, frame_off, n, lens, variant, stream=None):
    rx._check(_need(_tx_variant, "pn_tx_fill_variant")(ctx._h, rx._ptr(frames_dev), slot_stride, frame_off, n,
                                                       rx._ptr(lens), variant, rx._stream_handle(stream)),
              ctx._h, "pn_tx_fill_variant")
