"""ctypes mirror of the verify tile (include/fd_verify_tile.h,
firedancer_amd/csrc/fd_verify_tile.cpp) and of its HA dedup cache."""
from __future__ import annotations

import ctypes

import numpy as np

from . import EngineError, _p, last_error, lib

DIAG = ("IN_BACKP", "BACKP_CNT", "HA_FILT_CNT", "HA_FILT_SZ", "SV_FILT_CNT", "SV_FILT_SZ",
        "PUB_CNT", "PUB_SZ", "BAD_CNT", "SIG_CNT", "BATCH_CNT", "RING_FULL_CNT", "OVRN_CNT", "AGE_CNT")

PUBLISH_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_ulong,
                              ctypes.c_ulong, ctypes.c_ulong, ctypes.c_ulong)


class Cfg(ctypes.Structure):
    _fields_ = [("batch_sigs", ctypes.c_ulong), ("tcache_depth", ctypes.c_ulong), ("tcache_map_cnt", ctypes.c_ulong),
                ("max_wait_ns", ctypes.c_long)]


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


GPU_MAX = 8   # FD_VERIFY_TILE_GPU_MAX
LAT_BINS = 65536  # FD_VERIFY_TILE_LAT_BINS (1-us bins to 32.768 ms, then 64-us bins to 2.13 s)


def lat_bin_ms(b):
    """centre of native latency bin b, ms (fd_verify_tile_lat_publish)"""
    h = LAT_BINS // 2
    return (b + 0.5) * 1e-3 if b < h else (h + (b - h) * 64 + 32) * 1e-3


class LatHist:
    """fd_verify_tile_lat_t: a native publish callback's tsorig -> tspub
    histogram (fd_verify_tile_lat_publish), no Python per publish."""

    def __init__(self):
        self.buf = np.zeros(4 + LAT_BINS, np.uint64)

    @property
    def fn(self):
        return ctypes.cast(lib().fd_verify_tile_lat_publish, ctypes.c_void_p)

    @property
    def ctx(self):
        return self.buf.ctypes.data

    def reset(self):
        self.buf[:] = 0

    def summary(self) -> dict:
        cnt, sum_ns, max_ns, over = (int(x) for x in self.buf[:4])
        bins = self.buf[4:]
        if not cnt:
            return {"count": 0}
        c = np.cumsum(bins)

        def pct(q):
            return float(lat_bin_ms(int(np.searchsorted(c, q * cnt))))   # ms, bin centre

        return {"count": cnt, "mean_ms": sum_ns / cnt * 1e-6, "p50_ms": pct(0.5), "p99_ms": pct(0.99),
                "p999_ms": pct(0.999), "max_ms": max_ns * 1e-6, "over_2s": over}


class VerifyTile:
    """One verify tile on one Engine, or -- given a list of Engines -- on all
    of them in the multi-engine feeder mode (fd_verify_tile_new_multi).
    collect=True records every publish as (sig, frag bytes, ctl, tsorig);
    lat=LatHist() records tsorig -> tspub natively instead; otherwise
    publishes are only counted."""

    def __init__(self, engine, batch_sigs=0, tcache_depth=16, tcache_map_cnt=64, collect=True, lat=None, region=None,
                 max_wait_ns=0):
        """region (a contiguous uint8 array): the in-place mode
        (fd_verify_tile_new_inplace) -- every frag handed to rx_burst* lies
        in it and is DMA'd from where it lies, no copy; it must stay
        unchanged until the tile is flushed."""
        self.engine = engine
        self._region = region
        self.published = []
        self._cb = PUBLISH_FN(self._on_publish) if collect and lat is None else None
        cfg = Cfg(batch_sigs, tcache_depth, tcache_map_cnt, max_wait_ns)
        cb = ctypes.cast(self._cb, ctypes.c_void_p) if self._cb else None
        ctx = None
        if lat is not None:                       # native latency histogram (LatHist)
            cb, ctx = lat.fn, lat.ctx
            self._lat = lat
        if region is not None and (region.dtype != np.uint8 or not region.flags.c_contiguous):
            raise ValueError("region: a contiguous uint8 array")
        if isinstance(engine, (list, tuple)):
            L = lib()
            arr = (ctypes.c_void_p * len(engine))(*[e._h for e in engine])
            if region is not None:
                self._h = L.fd_verify_tile_new_multi_inplace(arr, len(engine), ctypes.byref(cfg), _p(region), region.nbytes,
                                                             cb, ctx)
            else:
                self._h = L.fd_verify_tile_new_multi(arr, len(engine), ctypes.byref(cfg), cb, ctx)
        elif region is not None:
            self._h = lib().fd_verify_tile_new_inplace(engine._h, ctypes.byref(cfg), _p(region), region.nbytes, cb, ctx)
        else:
            self._h = lib().fd_verify_tile_new(engine._h, ctypes.byref(cfg), cb, ctx)
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

    def rx_burst_now(self, base: np.ndarray, off: np.ndarray, sz: np.ndarray):
        """rx_burst with tsorig stamped at each frag's receipt"""
        off = np.ascontiguousarray(off, np.uint64)
        sz = np.ascontiguousarray(sz, np.uint32)
        err = lib().fd_verify_tile_rx_burst_now(self._h, _p(base), _p(off), _p(sz), len(off))
        if err:
            raise EngineError(f"rx_burst_now: {err}: {last_error()}")

    def held(self) -> int:
        """fd_verify_tile_held: receive index of the oldest frag still read"""
        return int(lib().fd_verify_tile_held(self._h))

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


# ---- the tile as a task (fd_verify_tile_task, include/fd_verify_tile.h) ----

SIGNAL_RUN, SIGNAL_BOOT, SIGNAL_FAIL, SIGNAL_HALT = 0, 1, 2, 3

IN_FN = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_ulong),
                         ctypes.POINTER(ctypes.c_ulong), ctypes.POINTER(ctypes.c_ulong))
CR_FN = ctypes.CFUNCTYPE(ctypes.c_ulong, ctypes.c_void_p)


class Cnc(ctypes.Structure):
    _fields_ = [("signal", ctypes.c_ulong), ("heartbeat", ctypes.c_long), ("diag", ctypes.c_ulong * len(DIAG))]


class Args(ctypes.Structure):
    """fd_verify_tile_args_t"""
    _fields_ = [("device", ctypes.c_int), ("max_sigs", ctypes.c_ulong), ("max_blob", ctypes.c_ulong),
                ("depth", ctypes.c_int), ("cfg", Cfg), ("cnc", ctypes.POINTER(Cnc)),
                ("in_fn", ctypes.c_void_p), ("in_ctx", ctypes.c_void_p),
                ("publish", ctypes.c_void_p), ("pub_ctx", ctypes.c_void_p),
                ("cr_avail", ctypes.c_void_p), ("cr_ctx", ctypes.c_void_p),
                ("lazy_ns", ctypes.c_long),
                ("close_fd_start", ctypes.c_uint), ("allow_syscalls_sz", ctypes.c_ushort),
                ("allow_syscalls", ctypes.POINTER(ctypes.c_long)),
                ("gpu", ctypes.c_void_p), ("tile", ctypes.c_void_p), ("err", ctypes.c_int),
                ("device_cnt", ctypes.c_int), ("gpus", ctypes.c_void_p * GPU_MAX),
                ("region", ctypes.c_void_p), ("region_sz", ctypes.c_ulong),
                ("in_seq", ctypes.c_void_p), ("ovrn", ctypes.c_void_p), ("chunk", ctypes.c_void_p),
                ("ovrn_ctx", ctypes.c_void_p), ("shared_gpu", ctypes.c_void_p)]


class TaskFns(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char_p), ("init", ctypes.c_void_p), ("run", ctypes.c_void_p), ("fini", ctypes.c_void_p)]


class Task:
    """fd_verify_tile_task driven from Python: frags from a list (the input
    mcache), publishes collected, optional credit schedule (the fctl).
    run() blocks until the cnc is signalled HALT (call halt() from
    another thread) or the task fails."""

    def __init__(self, frags, device=0, max_sigs=4096, max_blob=8 << 20, depth=3, batch_sigs=0,
                 credits=None, lazy_ns=0, device_cnt=0, max_wait_ns=0):
        L = lib()
        L.fd_verify_tile_task_get.restype = ctypes.POINTER(TaskFns)
        fns = L.fd_verify_tile_task_get().contents
        self.name = fns.name.decode()
        V = ctypes.CFUNCTYPE(None, ctypes.POINTER(Args))
        self._init, self._run, self._fini = V(fns.init), V(fns.run), V(fns.fini)
        self.frags = [ctypes.create_string_buffer(bytes(f), len(f)) for f in frags]
        self.sizes = [len(f) for f in frags]
        self.next = 0
        self.published = []
        self.credits = credits
        self.cnc = Cnc()
        self.cnc.signal = SIGNAL_BOOT
        self._in = IN_FN(self._on_in)
        self._pub = PUBLISH_FN(self._on_publish)
        self._cr = CR_FN(self._on_cr) if credits is not None else None
        a = Args()
        a.device, a.max_sigs, a.max_blob, a.depth = device, max_sigs, max_blob, depth
        a.cfg = Cfg(batch_sigs, 16, 64, max_wait_ns)
        a.cnc = ctypes.pointer(self.cnc)
        a.in_fn = ctypes.cast(self._in, ctypes.c_void_p)
        a.publish = ctypes.cast(self._pub, ctypes.c_void_p)
        a.cr_avail = ctypes.cast(self._cr, ctypes.c_void_p) if self._cr else None
        a.lazy_ns = lazy_ns
        a.device_cnt = device_cnt
        self.args = a

    def _on_in(self, ctx, frag, sz, ctl, tsorig):
        if self.next >= len(self.frags):
            return 0
        i = self.next
        self.next += 1
        frag[0] = ctypes.cast(self.frags[i], ctypes.c_void_p).value
        sz[0], ctl[0], tsorig[0] = self.sizes[i], i, 1000 + i
        return 1

    def _on_publish(self, ctx, sig, frag, sz, ctl, tsorig, tspub):
        self.published.append((sig, ctypes.string_at(frag, sz), ctl, tsorig))

    def _on_cr(self, ctx):
        return int(self.credits(self))

    def init(self):
        self._init(ctypes.byref(self.args))
        return self.args.err

    def allow_syscalls(self):
        return [self.args.allow_syscalls[i] for i in range(self.args.allow_syscalls_sz)]

    def run(self):
        self._run(ctypes.byref(self.args))
        return self.args.err

    def halt(self):
        self.cnc.signal = SIGNAL_HALT

    def diag(self) -> dict:
        return dict(zip(DIAG, list(self.cnc.diag)))

    def fini(self):
        self._fini(ctypes.byref(self.args))
