"""ctypes mirror of the verify tile (include/fd_verify_tile.h,
firedancer_amd/csrc/fd_verify_tile.cpp) and of its HA dedup cache."""
from __future__ import annotations

import ctypes

import numpy as np

from . import EngineError, _p, last_error, lib

DIAG = ("IN_BACKP", "BACKP_CNT", "HA_FILT_CNT", "HA_FILT_SZ", "SV_FILT_CNT", "SV_FILT_SZ",
        "PUB_CNT", "PUB_SZ", "BAD_CNT", "SIG_CNT", "BATCH_CNT")

PUBLISH_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_ulong,
                              ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong)


class Cfg(ctypes.Structure):
    _fields_ = [("batch_sigs", ctypes.c_ulong), ("tcache_depth", ctypes.c_ulong), ("tcache_map_cnt", ctypes.c_ulong)]


class TCache:
    """FD_TCACHE_INSERT semantics (src/tango/tcache/fd_tcache.h:373-400)."""

    def __init__(self, depth=16, map_cnt=64):
        self._h = lib().fd_vt_tcache_new(depth, map_cnt)
        if not self._h:
            raise ValueError("bad tcache geometry")

    def insert(self, tag: int) -> bool:
        return bool(lib().fd_vt_tcache_insert(self._h, tag))

    def close(self):
        if self._h:
            lib().fd_vt_tcache_delete(self._h)
            self._h = None

    __del__ = close


class VerifyTile:
    """One verify tile on one Engine.  collect=True records every publish
    as (sig, frag bytes, ctl, tsorig); otherwise publishes are only counted."""

    def __init__(self, engine, batch_sigs=0, tcache_depth=16, tcache_map_cnt=64, collect=True):
        self.engine = engine
        self.published = []
        self._cb = PUBLISH_FN(self._on_publish) if collect else None
        cfg = Cfg(batch_sigs, tcache_depth, tcache_map_cnt)
        self._h = lib().fd_verify_tile_new(engine._h, ctypes.byref(cfg),
                                           ctypes.cast(self._cb, ctypes.c_void_p) if self._cb else None, None)
        if not self._h:
            raise EngineError(f"fd_verify_tile_new failed: {last_error()}")

    def _on_publish(self, ctx, sig, frag, sz, ctl, tsorig, tspub):
        self.published.append((sig, ctypes.string_at(frag, sz), ctl, tsorig))

    def rx(self, frag: bytes, ctl=0, tsorig=0):
        buf = ctypes.create_string_buffer(frag, len(frag))
        err = lib().fd_verify_tile_rx(self._h, buf, len(frag), ctl, tsorig)
        if err:
            raise EngineError(f"rx: {err}: {last_error()}")

    def rx_burst(self, base: np.ndarray, off: np.ndarray, sz: np.ndarray, ctl=None, tsorig=None):
        off = np.ascontiguousarray(off, np.uint64)
        sz = np.ascontiguousarray(sz, np.uint32)
        c = _p(np.ascontiguousarray(ctl, np.uint64)) if ctl is not None else None
        t = _p(np.ascontiguousarray(tsorig, np.uint64)) if tsorig is not None else None
        err = lib().fd_verify_tile_rx_burst(self._h, _p(base), _p(off), _p(sz), c, t, len(off))
        if err:
            raise EngineError(f"rx_burst: {err}: {last_error()}")

    def service(self, flush=False):
        err = lib().fd_verify_tile_service(self._h, 1 if flush else 0)
        if err:
            raise EngineError(f"service: {err}: {last_error()}")

    def diag(self) -> dict:
        d = np.zeros(len(DIAG), np.uint64)
        lib().fd_verify_tile_diag(self._h, _p(d))
        return dict(zip(DIAG, d.tolist()))

    def close(self):
        if self._h:
            lib().fd_verify_tile_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
