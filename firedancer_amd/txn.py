"""Solana transaction wire format for the sigverify path.

Thin ctypes layer over the native parser in libfd_ed25519_gpu.so
(firedancer_amd/csrc/fd_txn_host.c, ABI include/fd_txn_abi.h), which
restates src/ballet/txn/fd_txn_parse.c:7-217 and writes the reference's
fd_txn_t byte layout (src/ballet/txn/fd_txn.h:107-320).

  parse(payload)      -> dict of fd_txn_t fields (+ 'instr', 'luts', 'footprint',
                         'raw' descriptor bytes) or None if malformed
  descs_for(payload)  -> one engine descriptor per signature: signature i over
                         the message with signer account i
                         (src/ballet/txn/fd_txn.h:159-217)
  frag(payload)       -> the QUIC tile's frag: payload | pad to 2 | fd_txn_t |
                         u16 payload_sz (src/disco/quic/fd_quic_tile.c:475-516)
"""
from __future__ import annotations

import ctypes
import struct

import numpy as np

from . import DESC_DTYPE, lib

TXN_MTU = 1232            # FD_TPU_MTU
SIG_MAX = 127             # FD_TXN_SIG_MAX, src/ballet/txn/fd_txn.h:65
ACCT_ADDR_MAX = 256       # FD_TXN_ACCT_ADDR_MAX, fd_txn.h:70
TXN_MAX_SZ = 3570         # FD_TXN_MAX_SZ, fd_txn.h:92
COUNTERS_RING_SZ = 32

_HDR = struct.Struct("<BBHHBBHHHBBBBH")        # fd_txn_t, 20 bytes
_INSTR = struct.Struct("<BBHHHH")              # fd_txn_instr_t, 10 bytes
_LUT = struct.Struct("<HBBHH")                 # fd_txn_acct_addr_lut_t, 8 bytes
_FIELDS = ("transaction_version", "signature_cnt", "signature_off", "message_off",
           "readonly_signed_cnt", "readonly_unsigned_cnt", "acct_addr_cnt", "acct_addr_off",
           "recent_blockhash_off", "addr_table_lookup_cnt", "addr_table_adtl_writable_cnt",
           "addr_table_adtl_cnt", "_padding_reserved_1", "instr_cnt")


class Counters(ctypes.Structure):
    """fd_txn_parse_counters_t (src/ballet/txn/fd_txn.h:326-341)."""
    _fields_ = [("success_cnt", ctypes.c_ulong), ("failure_cnt", ctypes.c_ulong),
                ("failure_ring", ctypes.c_ulong * COUNTERS_RING_SZ)]


def _fn():
    f = lib().fd_txn_parse
    f.argtypes = [ctypes.c_char_p, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]
    f.restype = ctypes.c_ulong
    return f


def parse_raw(payload: bytes, counters: Counters | None = None):
    """-> (footprint, descriptor bytes) with the native parser."""
    out = ctypes.create_string_buffer(TXN_MAX_SZ)
    fp = _fn()(bytes(payload), len(payload), out, ctypes.byref(counters) if counters is not None else None)
    return fp, out.raw[:fp]


def decode(raw: bytes) -> dict:
    t = dict(zip(_FIELDS, _HDR.unpack_from(raw, 0)))
    t["instr"] = [_INSTR.unpack_from(raw, 20 + 10 * j) for j in range(t["instr_cnt"])]
    lo = 20 + 10 * t["instr_cnt"]
    t["luts"] = [_LUT.unpack_from(raw, lo + 8 * j) for j in range(t["addr_table_lookup_cnt"])]
    t["footprint"] = len(raw)
    t["raw"] = raw
    return t


def parse(payload: bytes):
    fp, raw = parse_raw(payload)
    return decode(raw) if fp else None


def descs_for(payload: bytes, base: int = 0):
    """Engine descriptors for one txn placed at blob offset `base`."""
    t = parse(payload)
    if t is None:
        return None
    k = t["signature_cnt"]
    d = np.zeros(k, DESC_DTYPE)
    for j in range(k):
        d[j] = (base + t["signature_off"] + 64 * j, base + t["acct_addr_off"] + 32 * j,
                base + t["message_off"], len(payload) - t["message_off"])
    return d


def frag(payload: bytes):
    """QUIC-tile frag for a payload (None if it does not parse)."""
    fp, raw = parse_raw(payload)
    if not fp:
        return None
    pad = b"\x00" * (len(payload) & 1)
    return bytes(payload) + pad + raw + struct.pack("<H", len(payload))
