"""firedancer_amd -- MI355X-native Ed25519 signature verification engine.

Drop-in for tinydancer-io/firedancer's sigverify hot path
(``fd_ed25519_verify``, src/ballet/ed25519/fd_ed25519.h:96-101).  The
product is the C-ABI shared library ``libfd_ed25519_gpu.so`` (HIP kernels
for gfx950 + host runtime, declared in ``include/fd_ed25519_gpu.h``).
This module is a thin ctypes mirror of that ABI for tests, benchmarks
and Python callers; it never verifies anything itself and raises if the
library or a gfx950 device is missing.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("FD_ED25519_LIB") or os.path.join(_HERE, "libfd_ed25519_gpu.so")  # override: experiments only

SUCCESS = 0
ERR_SIG = -1
ERR_PUBKEY = -2
ERR_MSG = -3
ERR_ARG = -16
ERR_GPU = -17

MODE_AVX = 0        # reference AVX2 build semantics (default)
MODE_PORTABLE = 1   # reference FD_HAS_AVX=0 build semantics
MODE_STRICT = 2     # AVX checks with Q1-Q3 fixed (no reference build)


DESC_DTYPE = np.dtype([("sig_off", "<u4"), ("pub_off", "<u4"), ("msg_off", "<u4"), ("msg_sz", "<u4")])

_lib = None


class EngineError(RuntimeError):
    pass


def _share_hip_runtime():
    """One HIP runtime per process.  PyTorch-ROCm ships its own
    libamdhip64 (soname libamdhip64.so.7) and links it by file name, so if
    our library (which needs libamdhip64.so.7) were loaded first, torch
    would later load a second runtime and fail to initialise the GPU.
    Importing torch first makes the loader satisfy our dependency with
    torch's already-loaded copy.  Without torch, /opt/rocm's runtime is
    used."""
    if os.environ.get("FD_ED25519_NO_TORCH"):
        return
    try:
        import torch  # noqa: F401
    except Exception:
        pass


def lib() -> ctypes.CDLL:
    """Load the product library (fails loudly when it was not built)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise EngineError(f"{LIB_PATH} missing: run __graft_entry__.build() (make -C firedancer_amd)")
        _share_hip_runtime()
        L = ctypes.CDLL(LIB_PATH)
        vp, ul, ip = ctypes.c_void_p, ctypes.c_ulong, ctypes.c_int
        L.fd_ed25519_verify.argtypes = [vp, ul, vp, vp, vp]
        L.fd_ed25519_verify.restype = ip
        L.fd_ed25519_strerror.argtypes = [ip]
        L.fd_ed25519_strerror.restype = ctypes.c_char_p
        L.fd_ed25519_verify_batch.argtypes = [ul, vp, vp, vp, vp, vp]
        L.fd_ed25519_verify_batch.restype = ip
        L.fd_ed25519_verify_batch_single_msg.argtypes = [vp, ul, vp, vp, ul, vp]
        L.fd_ed25519_verify_batch_single_msg.restype = ip
        L.fd_ed25519_gpu_new.argtypes = [ip, ul, ul]
        L.fd_ed25519_gpu_new.restype = vp
        L.fd_ed25519_gpu_delete.argtypes = [vp]
        L.fd_ed25519_gpu_delete.restype = None
        L.fd_ed25519_gpu_verify_packed.argtypes = [vp, ul, vp, ul, vp, vp]
        L.fd_ed25519_gpu_verify_packed.restype = ip
        L.fd_ed25519_gpu_verify_dev.argtypes = [vp, ul, vp, ul, vp, vp, vp]
        L.fd_ed25519_gpu_verify_dev.restype = ip
        L.fd_ed25519_gpu_verify_dev_ex.argtypes = [vp, ul, vp, ul, vp, vp, vp, ip]
        L.fd_ed25519_gpu_verify_dev_ex.restype = ip
        L.fd_ed25519_gpu_verify_dev_timed.argtypes = [vp, ul, vp, ul, vp, vp, vp, vp]
        L.fd_ed25519_gpu_verify_dev_timed.restype = ip
        L.fd_ed25519_gpu_dev_stats_begin.argtypes = [vp]
        L.fd_ed25519_gpu_dev_stats_begin.restype = ip
        L.fd_ed25519_gpu_dev_stats_end.argtypes = [vp, vp, ctypes.POINTER(ctypes.c_ulong)]
        L.fd_ed25519_gpu_dev_stats_end.restype = ip
        L.fd_ed25519_gpu_dsm_clock.argtypes = [vp, ip, vp]
        L.fd_ed25519_gpu_dsm_clock.restype = ip
        L.fd_ed25519_gpu_kernel_cnt.argtypes = []
        L.fd_ed25519_gpu_kernel_cnt.restype = ip
        L.fd_ed25519_public_batch.argtypes = [ul, vp, vp, ip]
        L.fd_ed25519_public_batch.restype = None
        L.fd_ed25519_gpu_submit.argtypes = [vp, ul, vp, ul, vp, ctypes.POINTER(ctypes.c_ulong)]
        L.fd_ed25519_gpu_submit.restype = ip
        L.fd_ed25519_gpu_try_submit.argtypes = [vp, ul, vp, ul, vp, ctypes.POINTER(ctypes.c_ulong)]
        L.fd_ed25519_gpu_try_submit.restype = ip
        L.fd_ed25519_gpu_try_submit2.argtypes = [vp, ul, vp, ul, vp, ul, vp, ctypes.POINTER(ctypes.c_ulong)]
        L.fd_ed25519_gpu_try_submit2.restype = ip
        L.fd_ed25519_gpu_feeder_synth.argtypes = [vp, vp, ul, vp, ul, ul, vp, ul, ul, ip, ul, vp, vp]
        L.fd_ed25519_gpu_feeder_synth.restype = ip
        L.fd_ed25519_gpu_poll.argtypes = [vp, ul, vp, ip]
        L.fd_ed25519_gpu_poll.restype = ip
        L.fd_ed25519_gpu_depth.argtypes = [vp]
        L.fd_ed25519_gpu_depth.restype = ip
        L.fd_ed25519_gpu_set_timeout.argtypes = [vp, ctypes.c_long]
        L.fd_ed25519_gpu_set_timeout.restype = ip
        L.fd_ed25519_gpu_timeout.argtypes = [vp]
        L.fd_ed25519_gpu_timeout.restype = ctypes.c_long
        L.fd_ed25519_gpu_wait_selftest.argtypes = [ctypes.c_long, ctypes.c_long]
        L.fd_ed25519_gpu_wait_selftest.restype = ip
        L.fd_ed25519_gpu_device.argtypes = [vp]
        L.fd_ed25519_gpu_device.restype = ip
        L.fd_ed25519_gpu_last_error.argtypes = []
        L.fd_ed25519_gpu_last_error.restype = ctypes.c_char_p
        L.fd_ed25519_gpu_device_cnt.argtypes = []
        L.fd_ed25519_gpu_device_cnt.restype = ip
        L.fd_ed25519_public_from_private.argtypes = [vp, vp, vp]
        L.fd_ed25519_public_from_private.restype = vp
        L.fd_ed25519_sign.argtypes = [vp, vp, ul, vp, vp, vp]
        L.fd_ed25519_sign.restype = vp
        L.fd_ed25519_sign_batch.argtypes = [ul, vp, vp, vp, vp, vp, vp, ip]
        L.fd_ed25519_sign_batch.restype = None
        L.fd_ed25519_gpu_new_ex.argtypes = [ip, ul, ul, ip]
        L.fd_ed25519_gpu_new_ex.restype = vp
        L.fd_ed25519_gpu_max_sigs.argtypes = [vp]
        L.fd_ed25519_gpu_max_sigs.restype = ul
        L.fd_ed25519_gpu_max_blob.argtypes = [vp]
        L.fd_ed25519_gpu_max_blob.restype = ul
        L.fd_ed25519_gpu_verify_ptrs.argtypes = [vp, ul, vp, vp, vp, vp, vp]
        L.fd_ed25519_gpu_verify_ptrs.restype = ip
        L.fd_ed25519_gpu_stage.argtypes = [vp, ctypes.POINTER(vp), ctypes.POINTER(vp)]
        L.fd_ed25519_gpu_stage.restype = ip
        L.fd_ed25519_gpu_unstage.argtypes = [vp, vp]
        L.fd_ed25519_gpu_unstage.restype = None
        L.fd_txn_parse.argtypes = [vp, ul, vp, vp]
        L.fd_txn_parse.restype = ul
        L.fd_verify_tile_new.argtypes = [vp, vp, vp, vp]
        L.fd_verify_tile_new.restype = vp
        L.fd_verify_tile_delete.argtypes = [vp]
        L.fd_verify_tile_delete.restype = None
        L.fd_verify_tile_rx.argtypes = [vp, vp, ul, ul, ul]
        L.fd_verify_tile_rx.restype = ip
        L.fd_verify_tile_rx_burst.argtypes = [vp, vp, vp, vp, vp, vp, ul]
        L.fd_verify_tile_rx_burst.restype = ip
        L.fd_verify_tile_rx_burst_now.argtypes = [vp, vp, vp, vp, ul]
        L.fd_verify_tile_rx_burst_now.restype = ip
        L.fd_verify_tile_new_multi.argtypes = [vp, ul, vp, vp, vp]
        L.fd_verify_tile_new_multi.restype = vp
        L.fd_verify_tile_new_inplace.argtypes = [vp, vp, vp, ul, vp, vp]
        L.fd_verify_tile_new_inplace.restype = vp
        L.fd_verify_tile_new_multi_inplace.argtypes = [vp, ul, vp, vp, ul, vp, vp]
        L.fd_verify_tile_new_multi_inplace.restype = vp
        L.fd_verify_tile_held.argtypes = [vp]
        L.fd_verify_tile_held.restype = ul
        L.fd_verify_tile_service.argtypes = [vp, ip]
        L.fd_verify_tile_service.restype = ip
        L.fd_verify_tile_diag.argtypes = [vp, vp]
        L.fd_verify_tile_diag.restype = None
        L.fd_vt_tcache_new.argtypes = [ul, ul]
        L.fd_vt_tcache_new.restype = vp
        L.fd_vt_tcache_insert.argtypes = [vp, ul]
        L.fd_vt_tcache_insert.restype = ip
        L.fd_vt_tcache_delete.argtypes = [vp]
        L.fd_vt_tcache_delete.restype = None
        L.fd_ed25519_gpu_debug_k.argtypes = [vp, ul, vp, ul, vp, vp, vp]
        L.fd_ed25519_gpu_debug_k.restype = ip
        L.fd_ed25519_gpu_debug_fe.argtypes = [vp, ip, ul, vp, vp, vp]
        L.fd_ed25519_gpu_debug_fe.restype = ip
        L.fd_ed25519_gpu_sha512_packed.argtypes = [vp, ul, vp, ul, vp, vp, ip]
        L.fd_ed25519_gpu_sha512_packed.restype = ip
        L.fd_ed25519_gpu_default.argtypes = []
        L.fd_ed25519_gpu_default.restype = vp
        L.fd_ed25519_gpu_set_mode.argtypes = [vp, ip]
        L.fd_ed25519_gpu_set_mode.restype = ip
        L.fd_ed25519_gpu_mode.argtypes = [vp]
        L.fd_ed25519_gpu_mode.restype = ip
        L.fd_ed25519_gpu_set_dsm_pool_min.argtypes = [vp, ul]
        L.fd_ed25519_gpu_set_dsm_pool_min.restype = ip
        L.fd_ed25519_gpu_dsm_pool_min.argtypes = [vp]
        L.fd_ed25519_gpu_dsm_pool_min.restype = ul
        L.fd_ed25519_gpu_set_dsm_quad_max.argtypes = [vp, ul]
        L.fd_ed25519_gpu_set_dsm_quad_max.restype = ip
        L.fd_ed25519_gpu_dsm_quad_max.argtypes = [vp]
        L.fd_ed25519_gpu_dsm_quad_max.restype = ul
        L.fd_ed25519_gpu_set_dsm_oct_max.argtypes = [vp, ul]
        L.fd_ed25519_gpu_set_dsm_oct_max.restype = ip
        L.fd_ed25519_gpu_dsm_oct_max.argtypes = [vp]
        L.fd_ed25519_gpu_dsm_oct_max.restype = ul
        L.fd_ed25519_gpu_multi_new.argtypes = [vp, ip, ul, ul]
        L.fd_ed25519_gpu_multi_new.restype = vp
        L.fd_ed25519_gpu_multi_delete.argtypes = [vp]
        L.fd_ed25519_gpu_multi_delete.restype = None
        L.fd_ed25519_gpu_multi_cnt.argtypes = [vp]
        L.fd_ed25519_gpu_multi_cnt.restype = ip
        L.fd_ed25519_gpu_multi_engine.argtypes = [vp, ip]
        L.fd_ed25519_gpu_multi_engine.restype = vp
        L.fd_ed25519_gpu_multi_verify_packed.argtypes = [vp, ul, vp, ul, vp, vp]
        L.fd_ed25519_gpu_multi_verify_packed.restype = ip
        L.fd_ed25519_codes_to_bitmap.argtypes = [ul, vp, vp]
        L.fd_ed25519_codes_to_bitmap.restype = None
        L.fd_ed25519_gpu_set_cu_groups.argtypes = [vp, ip]
        L.fd_ed25519_gpu_set_cu_groups.restype = ip
        L.fd_ed25519_gpu_cu_groups.argtypes = [vp]
        L.fd_ed25519_gpu_cu_groups.restype = ip
        L.fd_ed25519_gpu_register.argtypes = [vp, vp, ul]
        L.fd_ed25519_gpu_register.restype = ip
        L.fd_ed25519_gpu_unregister.argtypes = [vp, vp]
        L.fd_ed25519_gpu_unregister.restype = ip
        L.fd_ed25519_gpu_feeder_new.argtypes = [vp, ip]
        L.fd_ed25519_gpu_feeder_new.restype = vp
        L.fd_ed25519_gpu_feeder_delete.argtypes = [vp]
        L.fd_ed25519_gpu_feeder_delete.restype = None
        L.fd_ed25519_gpu_device_numa_node.argtypes = [ip]
        L.fd_ed25519_gpu_device_numa_node.restype = ip
        L.fd_ed25519_gpu_feeder_numa_node.argtypes = [vp]
        L.fd_ed25519_gpu_feeder_numa_node.restype = ip
        L.fd_ed25519_gpu_feeder_push.argtypes = [vp, vp]
        L.fd_ed25519_gpu_feeder_push.restype = ip
        L.fd_ed25519_gpu_job_wait.argtypes = [vp, ctypes.c_long]
        L.fd_ed25519_gpu_job_wait.restype = ip
        L.fd_ed25519_gpu_multi_new_ex.argtypes = [vp, ip, ul, ul, ip]
        L.fd_ed25519_gpu_multi_new_ex.restype = vp
        L.fd_ed25519_gpu_multi_feeder.argtypes = [vp, ip]
        L.fd_ed25519_gpu_multi_feeder.restype = vp
        L.fd_sha512_gpu_batch_new.argtypes = [vp, ip]
        L.fd_sha512_gpu_batch_new.restype = vp
        L.fd_sha512_gpu_batch_delete.argtypes = [vp]
        L.fd_sha512_gpu_batch_delete.restype = None
        L.fd_sha512_gpu_batch_init.argtypes = [vp]
        L.fd_sha512_gpu_batch_init.restype = vp
        L.fd_sha512_gpu_batch_add.argtypes = [vp, vp, ul, vp]
        L.fd_sha512_gpu_batch_add.restype = vp
        L.fd_sha512_gpu_batch_fini.argtypes = [vp]
        L.fd_sha512_gpu_batch_fini.restype = vp
        L.fd_sha512_gpu_batch_abort.argtypes = [vp]
        L.fd_sha512_gpu_batch_abort.restype = vp
        _lib = L
    return _lib


def _p(a: np.ndarray) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def strerror(err: int) -> str:
    return lib().fd_ed25519_strerror(err).decode()


def last_error() -> str:
    return (lib().fd_ed25519_gpu_last_error() or b"").decode()


class Engine:
    """One verification engine bound to one gfx950 device (fd_ed25519_gpu_t)."""

    def __init__(self, device: int = 0, max_sigs: int = 1 << 16, max_blob: int = 1 << 26, depth: int = 3):
        L = lib()
        self._h = L.fd_ed25519_gpu_new_ex(device, max_sigs, max_blob, depth)
        if not self._h:
            raise EngineError(f"fd_ed25519_gpu_new(device={device}) failed: {last_error()}")
        self.device = device
        self.max_sigs = max_sigs
        self.max_blob = max_blob
        self._pending = {}
        self._registered = []

    def close(self):
        if self._h:
            lib().fd_ed25519_gpu_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def verify_packed(self, blob: np.ndarray, desc: np.ndarray) -> np.ndarray:
        """Host batch in, host codes out (synchronous)."""
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        out = np.empty(len(desc), dtype=np.int32)
        err = lib().fd_ed25519_gpu_verify_packed(self._h, len(desc), _p(blob), blob.nbytes, _p(desc), _p(out))
        if err:
            raise EngineError(f"verify_packed: {strerror(err)}: {last_error()}")
        return out

    def verify_ptrs(self, msgs, sigs, pubs) -> tuple[int, np.ndarray]:
        """fd_ed25519_gpu_verify_ptrs: fd_ed25519_verify_batch on this engine,
        messages of any length (past max_blob: the long path)."""
        n = len(msgs)
        keep = [m if isinstance(m, np.ndarray) else np.frombuffer(bytes(m), np.uint8) for m in msgs]
        sb = [ctypes.create_string_buffer(bytes(x), 64) for x in sigs]
        pb = [ctypes.create_string_buffer(bytes(x), 32) for x in pubs]
        MP = ctypes.c_void_p * max(n, 1)
        mp = MP(*[m.ctypes.data if len(m) else None for m in keep])
        sp = MP(*[ctypes.cast(b, ctypes.c_void_p) for b in sb])
        pp = MP(*[ctypes.cast(b, ctypes.c_void_p) for b in pb])
        sz = (ctypes.c_ulong * max(n, 1))(*[len(m) for m in keep])
        out = np.zeros(n, dtype=np.int32)
        r = lib().fd_ed25519_gpu_verify_ptrs(self._h, n, mp, sz, sp, pp, _p(out))
        if r in (ERR_ARG, ERR_GPU):
            raise EngineError(f"verify_ptrs: {strerror(r)}: {last_error()}")
        return r, out

    def verify_dev(self, n: int, d_blob: int, blob_sz: int, d_desc: int, d_out: int, stream: int = 0,
                   inputs_ready: bool = False) -> None:
        """Device-resident batch (raw device pointers, e.g. torch tensor .data_ptr());
        blob_sz = payload bytes at d_blob (descriptors are bounds-checked against it).
        inputs_ready: the inputs are already complete on the device (no ordering
        after work queued on `stream`), so successive launches overlap."""
        err = lib().fd_ed25519_gpu_verify_dev_ex(self._h, n, d_blob, blob_sz, d_desc, d_out, stream or None,
                                                 1 if inputs_ready else 0)
        if err:
            raise EngineError(f"verify_dev: {strerror(err)}: {last_error()}")

    KERNELS = ("fd_k_prep", "fd_k_decomp", "fd_k_dsm_setup", "fd_k_dsm_pool", "fd_k_dsm_final")

    def verify_dev_timed(self, n: int, d_blob: int, blob_sz: int, d_desc: int, d_out: int, stream: int = 0) -> np.ndarray:
        """verify_dev with per-kernel HIP-event durations (ms), in KERNELS order."""
        ms = np.zeros(lib().fd_ed25519_gpu_kernel_cnt(), np.float32)
        err = lib().fd_ed25519_gpu_verify_dev_timed(self._h, n, d_blob, blob_sz, d_desc, d_out, stream or None, _p(ms))
        if err:
            raise EngineError(f"verify_dev_timed: {strerror(err)}: {last_error()}")
        return ms

    def dev_stats_begin(self) -> None:
        """start timing each kernel of the following pipelined verify_dev launches"""
        if lib().fd_ed25519_gpu_dev_stats_begin(self._h):
            raise EngineError("dev_stats_begin")

    def dev_stats_end(self):
        """-> (per-kernel mean ms over the launches since begin, in KERNELS order; launches)"""
        ms = np.zeros(lib().fd_ed25519_gpu_kernel_cnt(), np.float32)
        cnt = ctypes.c_ulong(0)
        err = lib().fd_ed25519_gpu_dev_stats_end(self._h, _p(ms), ctypes.byref(cnt))
        if err:
            raise EngineError(f"dev_stats_end: {strerror(err)}: {last_error()}")
        return (ms / max(cnt.value, 1)).astype(np.float64), cnt.value

    def dsm_clock(self, clear: bool = False):
        """Shader clock the DSM kernels ran at on this engine's device since
        the last clear (fd_ed25519_gpu_dsm_clock): None after clear=True,
        else {"pool": {"waves", "ghz"}, "quad": {...}, "oct": {...}} (ghz None when no wave
        of that kernel ran).  Call with the device idle."""
        out = np.zeros(9, np.uint64)
        err = lib().fd_ed25519_gpu_dsm_clock(self._h, 1 if clear else 0, None if clear else _p(out))
        if err:
            raise EngineError(f"dsm_clock: {strerror(err)}: {last_error()}")
        if clear:
            return None
        def one(w, c, t):
            return {"waves": int(w), "ghz": (0.1 * float(c) / float(t)) if t else None,
                    "cycles_per_wave": float(c) / float(w) if w else None,
                    "us_per_wave": 0.01 * float(t) / float(w) if w else None}
        return {"pool": one(*out[0:3]), "quad": one(*out[3:6]), "oct": one(*out[6:9])}

    def submit(self, blob: np.ndarray, desc: np.ndarray) -> int:
        """Queue a batch on the pinned ring; returns its ticket."""
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        t = ctypes.c_ulong(0)
        err = lib().fd_ed25519_gpu_submit(self._h, len(desc), _p(blob), blob.nbytes, _p(desc), ctypes.byref(t))
        if err:
            raise EngineError(f"submit: {strerror(err)}: {last_error()}")
        self._pending[t.value] = len(desc)
        return t.value

    def poll(self, ticket: int, out: np.ndarray, block: bool = True) -> bool:
        """Collect a ticket's codes into out (int32, contiguous, >= the batch's
        signature count); False while the batch is in flight."""
        n = self._pending.get(ticket)
        if n is None:
            raise EngineError(f"poll: unknown ticket {ticket}")
        if not isinstance(out, np.ndarray) or out.dtype != np.int32 or not out.flags.c_contiguous or out.size < n:
            raise EngineError(f"poll: out must be a contiguous int32 array of >= {n} entries")
        r = lib().fd_ed25519_gpu_poll(self._h, ticket, _p(out), 1 if block else 0)
        if r < 0:
            raise EngineError(f"poll: {strerror(r)}: {last_error()}")
        if r == 1:
            del self._pending[ticket]
        return r == 1

    @property
    def timeout_ns(self) -> int:
        """bound on one blocking wait (ns; < 0 unbounded)"""
        return lib().fd_ed25519_gpu_timeout(self._h)

    @timeout_ns.setter
    def timeout_ns(self, ns: int) -> None:
        if lib().fd_ed25519_gpu_set_timeout(self._h, int(ns)):
            raise EngineError("set_timeout")

    def debug_k(self, blob: np.ndarray, desc: np.ndarray):
        """Diagnostics: (k[n,32], status[n]) from fd_k_prep -- k = SHA-512(R||A||M)
        mod L for signatures whose S check is pending (status 1), else zeros."""
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        k = np.zeros((len(desc), 32), np.uint8)
        st = np.zeros(len(desc), np.int32)
        err = lib().fd_ed25519_gpu_debug_k(self._h, len(desc), _p(blob), blob.nbytes, _p(desc), _p(k), _p(st))
        if err:
            raise EngineError(f"debug_k: {strerror(err)}: {last_error()}")
        return k, st

    def debug_fe(self, op: int, f: np.ndarray, g: np.ndarray) -> np.ndarray:
        """Diagnostics: the device field products (fd_k_debug_fe op 0-6, op 7 the oct DSM's half product) of
        operand pairs f, g ([n,10] int32 limbs) -> [3,n,10] int32 limbs."""
        f = np.ascontiguousarray(f, dtype=np.int32).reshape(-1, 10)
        g = np.ascontiguousarray(g, dtype=np.int32).reshape(-1, 10)
        if f.shape != g.shape:
            raise EngineError("debug_fe: f and g differ in shape")
        h = np.zeros((3, len(f), 10), np.int32)
        err = lib().fd_ed25519_gpu_debug_fe(self._h, int(op), len(f), _p(f), _p(g), _p(h))
        if err:
            raise EngineError(f"debug_fe: {strerror(err)}: {last_error()}")
        return h

    def sha512(self, msgs, is384: bool = False) -> list:
        """SHA-512 (SHA-384) digests of byte strings on the device."""
        n = len(msgs)
        if n == 0:
            return []
        offs, parts, o = [], [], 0
        for m in msgs:
            offs.append(o)
            parts.append(bytes(m) + b"\0" * ((-len(m)) % 8))
            o += len(parts[-1])
        blob = np.frombuffer(b"".join(parts) + b"\0", np.uint8).copy()
        desc = np.zeros(n, DESC_DTYPE)
        desc["msg_off"] = offs
        desc["msg_sz"] = [len(m) for m in msgs]
        hsz = 48 if is384 else 64
        out = np.zeros(n * hsz, np.uint8)
        err = lib().fd_ed25519_gpu_sha512_packed(self._h, n, _p(blob), o, _p(desc), _p(out), 1 if is384 else 0)
        if err:
            raise EngineError(f"sha512_packed: {strerror(err)}: {last_error()}")
        return [out[i * hsz:(i + 1) * hsz].tobytes() for i in range(n)]

    @property
    def mode(self) -> int:
        return lib().fd_ed25519_gpu_mode(self._h)

    @mode.setter
    def mode(self, m: int) -> None:
        if lib().fd_ed25519_gpu_set_mode(self._h, m):
            raise EngineError(f"bad mode {m}")

    @property
    def dsm_pool_min(self) -> int:
        """batches of at least this many signatures take the pooled DSM"""
        return lib().fd_ed25519_gpu_dsm_pool_min(self._h)

    @dsm_pool_min.setter
    def dsm_pool_min(self, n: int) -> None:
        if lib().fd_ed25519_gpu_set_dsm_pool_min(self._h, n):
            raise EngineError("set_dsm_pool_min")

    @property
    def dsm_quad_max(self) -> int:
        """smaller batches of at most this many signatures take the quad-lane DSM"""
        return lib().fd_ed25519_gpu_dsm_quad_max(self._h)

    @dsm_quad_max.setter
    def dsm_quad_max(self, n: int) -> None:
        if lib().fd_ed25519_gpu_set_dsm_quad_max(self._h, n):
            raise EngineError("set_dsm_quad_max")

    @property
    def dsm_oct_max(self) -> int:
        """batches of at most this many signatures (below dsm_pool_min) run the eight-lane DSM"""
        return lib().fd_ed25519_gpu_dsm_oct_max(self._h)

    @dsm_oct_max.setter
    def dsm_oct_max(self, n: int) -> None:
        if lib().fd_ed25519_gpu_set_dsm_oct_max(self._h, n):
            raise EngineError("set_dsm_oct_max")

    @property
    def depth(self) -> int:
        return lib().fd_ed25519_gpu_depth(self._h)

    @property
    def cu_groups(self) -> int:
        """CU groups the ring's small batches are spread over (1: none)"""
        return lib().fd_ed25519_gpu_cu_groups(self._h)

    @cu_groups.setter
    def cu_groups(self, g: int) -> None:
        if lib().fd_ed25519_gpu_set_cu_groups(self._h, int(g)):
            raise EngineError(f"set_cu_groups({g}): ring busy or bad count")

    def register(self, host: np.ndarray) -> None:
        """Let the ring DMA batches straight from this (contiguous) host array."""
        if not host.flags.c_contiguous:
            raise EngineError("register: array must be contiguous")
        if lib().fd_ed25519_gpu_register(self._h, _p(host), host.nbytes):
            raise EngineError(f"register: {last_error()}")
        self._registered.append(host)

    def unregister(self, host: np.ndarray) -> None:
        if lib().fd_ed25519_gpu_unregister(self._h, _p(host)):
            raise EngineError(f"unregister: {last_error()}")
        self._registered = [a for a in self._registered if a is not host]


class Job(ctypes.Structure):
    """fd_ed25519_gpu_job_t"""
    _fields_ = [("n", ctypes.c_ulong), ("blob", ctypes.c_void_p), ("blob_sz", ctypes.c_ulong),
                ("desc", ctypes.c_void_p), ("out", ctypes.c_void_p), ("state", ctypes.c_int),
                ("t_push_ns", ctypes.c_ulong), ("t_submit_ns", ctypes.c_ulong), ("t_done_ns", ctypes.c_ulong),
                ("t_pick_ns", ctypes.c_ulong), ("blob2", ctypes.c_void_p), ("blob2_sz", ctypes.c_ulong)]


# fd_ed25519_gpu_synth_stat_t
SYNTH_STAT_DTYPE = np.dtype([("t_sched_ns", "<u8"), ("t_push_ns", "<u8"), ("t_submit_ns", "<u8"), ("t_done_ns", "<u8"),
                             ("t_pick_ns", "<u8"), ("state", "<i4"), ("codes", "<u4", (5,))], align=True)


class Feeder:
    """The per-GPU feeder thread (fd_ed25519_gpu_feeder_t) over an Engine's ring."""

    def __init__(self, engine: Engine, pin_numa: bool = True):
        self.engine = engine
        self._h = lib().fd_ed25519_gpu_feeder_new(engine._h, 1 if pin_numa else 0)
        if not self._h:
            raise EngineError("fd_ed25519_gpu_feeder_new failed")
        self._keep = {}

    @property
    def numa_node(self) -> int:
        return lib().fd_ed25519_gpu_feeder_numa_node(self._h)

    def push(self, blob: np.ndarray, desc: np.ndarray, out: np.ndarray, job: Job = None) -> Job:
        """Queue a batch; the arrays must stay alive and unchanged until the job completes."""
        if blob.dtype != np.uint8 or not blob.flags.c_contiguous or desc.dtype != DESC_DTYPE or not desc.flags.c_contiguous:
            raise EngineError("push: contiguous uint8 blob and DESC_DTYPE desc required")
        if out.dtype != np.int32 or not out.flags.c_contiguous or out.size < len(desc):
            raise EngineError("push: out must be a contiguous int32 array of >= len(desc) entries")
        j = job if job is not None else Job()
        j.n, j.blob, j.blob_sz, j.desc, j.out = len(desc), blob.ctypes.data, blob.nbytes, desc.ctypes.data, out.ctypes.data
        self._keep[ctypes.addressof(j)] = (blob, desc, out)
        err = lib().fd_ed25519_gpu_feeder_push(self._h, ctypes.byref(j))
        if err:
            raise EngineError(f"feeder push: {strerror(err)}")
        return j

    def wait(self, job: Job, timeout_ns: int = -1) -> None:
        err = lib().fd_ed25519_gpu_job_wait(ctypes.byref(job), timeout_ns)
        # the arrays stay referenced until the job reached a final state: after
        # a timeout it is still queued or in flight on the feeder thread, which
        # may yet read the blob and descriptors and write the codes
        # (close() releases them once the feeder has drained)
        if job.state != 0:
            self._keep.pop(ctypes.addressof(job), None)
        if err:
            raise EngineError(f"job: {strerror(err)}: {last_error()}")

    def synth(self, blob: np.ndarray, desc: np.ndarray, batch_sigs: int, starts, nbatch: int, window: int,
              period_ns: int = 0, codes: bool = False):
        """The native synthetic-load producer (fd_ed25519_gpu_feeder_synth): nbatch
        jobs of batch_sigs signatures, job i from desc[starts[i % len(starts)]:],
        closed loop with `window` outstanding (period_ns 0) or paced one job per
        period_ns.  Returns the per-job SYNTH_STAT_DTYPE records, and with
        codes=True also every code as int8 [nbatch, batch_sigs]."""
        blob = np.ascontiguousarray(blob, np.uint8)
        desc = np.ascontiguousarray(desc, DESC_DTYPE)
        st = np.ascontiguousarray(starts, np.uint64)
        stat = np.zeros(nbatch, SYNTH_STAT_DTYPE)
        cs = np.full((nbatch, batch_sigs), 99, np.int8) if codes else None
        err = lib().fd_ed25519_gpu_feeder_synth(self._h, _p(blob), blob.nbytes, _p(desc), len(desc), batch_sigs,
                                                _p(st), len(st), nbatch, window, period_ns, _p(stat),
                                                _p(cs) if codes else None)
        if err:
            raise EngineError(f"feeder synth: {strerror(err)}: {last_error()}")
        return (stat, cs) if codes else stat

    def close(self):
        if self._h:
            lib().fd_ed25519_gpu_feeder_delete(self._h)
            self._h = None
            self._keep.clear()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MultiEngine:
    """Engines on several devices (repeats allowed) behind one host:
    fd_ed25519_gpu_multi_t."""

    def __init__(self, devices, max_sigs: int = 1 << 16, max_blob: int = 1 << 26, depth: int = 3):
        d = np.ascontiguousarray(devices, np.int32)
        self._h = lib().fd_ed25519_gpu_multi_new_ex(_p(d), len(d), max_sigs, max_blob, depth)
        if not self._h:
            raise EngineError(f"fd_ed25519_gpu_multi_new({list(devices)}) failed: {last_error()}")

    def verify_packed(self, blob: np.ndarray, desc: np.ndarray) -> np.ndarray:
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        out = np.empty(len(desc), dtype=np.int32)
        err = lib().fd_ed25519_gpu_multi_verify_packed(self._h, len(desc), _p(blob), blob.nbytes, _p(desc), _p(out))
        if err:
            raise EngineError(f"multi verify_packed: {strerror(err)}: {last_error()}")
        return out

    @property
    def count(self) -> int:
        return lib().fd_ed25519_gpu_multi_cnt(self._h)

    def close(self):
        if self._h:
            lib().fd_ed25519_gpu_multi_delete(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def codes_to_bitmap(codes: np.ndarray) -> np.ndarray:
    codes = np.ascontiguousarray(codes, np.int32)
    bm = np.zeros((len(codes) + 7) // 8, np.uint8)
    lib().fd_ed25519_codes_to_bitmap(len(codes), _p(codes), _p(bm))
    return bm


def verify(msg: bytes, sig: bytes, pub: bytes) -> int:
    """fd_ed25519_verify on the process-default engine."""
    m = ctypes.create_string_buffer(bytes(msg), max(1, len(msg)))
    s = ctypes.create_string_buffer(bytes(sig), 64)
    p = ctypes.create_string_buffer(bytes(pub), 32)
    return lib().fd_ed25519_verify(m, len(msg), s, p, None)


def verify_batch(msgs, sigs, pubs) -> tuple[int, np.ndarray]:
    """fd_ed25519_verify_batch over Python byte strings."""
    n = len(msgs)
    bufs = [ctypes.create_string_buffer(bytes(m), max(1, len(m))) for m in msgs]
    sb = [ctypes.create_string_buffer(bytes(s), 64) for s in sigs]
    pb = [ctypes.create_string_buffer(bytes(p), 32) for p in pubs]
    MP = ctypes.c_void_p * n
    mp = MP(*[ctypes.cast(b, ctypes.c_void_p) for b in bufs])
    sp = MP(*[ctypes.cast(b, ctypes.c_void_p) for b in sb])
    pp = MP(*[ctypes.cast(b, ctypes.c_void_p) for b in pb])
    sz = (ctypes.c_ulong * n)(*[len(m) for m in msgs])
    out = np.zeros(n, dtype=np.int32)
    r = lib().fd_ed25519_verify_batch(n, mp, sz, sp, pp, _p(out))
    return r, out


def verify_batch_single_msg(msg: bytes, sigs: np.ndarray, pubs: np.ndarray) -> tuple[int, np.ndarray]:
    sigs = np.ascontiguousarray(sigs, dtype=np.uint8).reshape(-1, 64)
    pubs = np.ascontiguousarray(pubs, dtype=np.uint8).reshape(-1, 32)
    n = len(sigs)
    m = ctypes.create_string_buffer(bytes(msg), max(1, len(msg)))
    out = np.zeros(n, dtype=np.int32)
    r = lib().fd_ed25519_verify_batch_single_msg(m, len(msg), _p(sigs), _p(pubs), n, _p(out))
    return r, out


def device_count() -> int:
    return lib().fd_ed25519_gpu_device_cnt()


def kernels_id() -> str:
    """build id of the loaded library's device code (fd_ed25519_gpu_kernels_id)"""
    f = lib().fd_ed25519_gpu_kernels_id
    f.restype = ctypes.c_char_p
    return f().decode()


def numa_cpus(device: int) -> list:
    """CPUs of the device's NUMA node this process may use ([] if unknown)."""
    node = lib().fd_ed25519_gpu_device_numa_node(device)
    if node < 0:
        return []
    cpus = set()
    for part in open(f"/sys/devices/system/node/node{node}/cpulist").read().strip().split(","):
        lo, _, hi = part.partition("-")
        cpus.update(range(int(lo), int(hi or lo) + 1))
    return sorted(cpus & os.sched_getaffinity(0))


def _cpu_times() -> dict:
    out = {}
    for line in open("/proc/stat"):
        if line.startswith("cpu") and line[3].isdigit():
            f = line.split()
            v = [int(x) for x in f[1:]]
            out[int(f[0][3:])] = (v[3] + (v[4] if len(v) > 4 else 0), sum(v))   # (idle + iowait, total)
    return out


def _core_siblings(c: int) -> set:
    try:
        txt = open(f"/sys/devices/system/cpu/cpu{c}/topology/thread_siblings_list").read().strip()
    except OSError:
        return {c}
    sib = set()
    for part in txt.split(","):
        lo, _, hi = part.partition("-")
        sib.update(range(int(lo), int(hi or lo) + 1))
    return sib


def _l3_group(c: int) -> str:
    try:
        return open(f"/sys/devices/system/cpu/cpu{c}/cache/index3/shared_cpu_list").read().strip()
    except OSError:
        return ""


def quiet_cpus(n: int, device: int = 0, sample_s: float = 0.3, pairs: bool = True) -> list:
    """n CPUs for spinning host threads (tiles, feeders, producers): on the
    device's NUMA node, not CPU 0, one per physical core, the least busy over
    a short /proc/stat sample counting each core's other hardware threads --
    on a shared host other work lands on some CPUs, and a spinning thread
    that shares its core with it stalls for milliseconds.  pairs: CPUs
    2k and 2k+1 (a producer and its consumer) share a last-level cache, so
    the bytes one writes reach the other without crossing chiplets (on the
    GPU box's EPYC one CCD of 8 cores per L3).  [] if that many cannot be
    found."""
    import time
    cand = [c for c in (numa_cpus(device) or sorted(os.sched_getaffinity(0))) if c != 0]
    if len(cand) < n:
        return []
    t0 = _cpu_times()
    time.sleep(sample_s)
    t1 = _cpu_times()

    def busy(c):
        if c not in t0 or c not in t1 or t1[c][1] <= t0[c][1]:
            return 0.0
        return 1.0 - (t1[c][0] - t0[c][0]) / (t1[c][1] - t0[c][1])
    score = {c: sum(busy(x) for x in _core_siblings(c)) for c in cand}
    order = sorted(cand, key=lambda c: (score[c], c))
    pick, used = [], set()
    if pairs and n >= 2:
        # quietest pairs first, each pair from one L3 group
        while len(pick) + 2 <= n:
            best = None
            groups = {}
            for c in order:
                if c in used:
                    continue
                groups.setdefault(_l3_group(c), []).append(c)
            for g, cs in groups.items():
                two = []
                seen = set()
                for c in cs:                          # one per physical core
                    if c in seen:
                        continue
                    two.append(c)
                    seen |= _core_siblings(c)
                    if len(two) == 2:
                        break
                if len(two) == 2 and (best is None or score[two[0]] + score[two[1]] < best[0]):
                    best = (score[two[0]] + score[two[1]], two)
            if best is None:
                break
            for c in best[1]:
                pick.append(c)
                used |= _core_siblings(c)
        if len(pick) == n:
            return pick
        if len(pick) + 1 != n:
            pick, used = [], set()
    for c in order:
        if c in used:
            continue
        pick.append(c)
        used |= _core_siblings(c)
        if len(pick) == n:
            return pick
    return []


def sign_batch(seeds: np.ndarray, blob: np.ndarray, msg_off: np.ndarray, msg_sz: np.ndarray, nthreads: int = 8):
    """Host signer (test-data generation only): returns (pub[n,32], sig[n,64])."""
    seeds = np.ascontiguousarray(seeds, dtype=np.uint8).reshape(-1, 32)
    n = len(seeds)
    blob = np.ascontiguousarray(blob, dtype=np.uint8)
    msg_off = np.ascontiguousarray(msg_off, dtype=np.uint64)
    msg_sz = np.ascontiguousarray(msg_sz, dtype=np.uint32)
    pub = np.zeros((n, 32), np.uint8)
    sig = np.zeros((n, 64), np.uint8)
    lib().fd_ed25519_sign_batch(n, _p(seeds), _p(blob), _p(msg_off), _p(msg_sz), _p(pub), _p(sig), nthreads)
    return pub, sig
