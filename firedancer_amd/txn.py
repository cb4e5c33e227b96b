"""Minimal Solana transaction wire parsing for the sigverify path.

Mirrors the parts of fd_txn_parse (src/ballet/txn/fd_txn_parse.c, layout
in src/ballet/txn/fd_txn.h:159-217) that the verify tile needs: the
signature count, the offsets of the signatures, of the signer account
addresses and of the message.  Each transaction yields signature_cnt
(sig_i, pub_i, msg) tuples with sig_i = payload[sig_off + 64 i],
pub_i = payload[acct_off + 32 i], msg = payload[msg_off:]
(src/wiredancer/test/test_wiredancer_demo.c:364-370).  Malformed input
returns None (the reference drops such txns before verify).
"""
from __future__ import annotations

import numpy as np

from . import DESC_DTYPE

TXN_MTU = 1232
SIG_MAX = 12  # FD_TXN_SIG_MAX, src/ballet/txn/fd_txn.h:55-57
ACCT_ADDR_MAX = 128


def _cu16(b, i):
    """compact-u16 decode -> (value, next index) or None."""
    v = 0
    for k in range(3):
        if i + k >= len(b):
            return None
        c = b[i + k]
        if k == 2 and c > 3:
            return None
        v |= (c & 0x7F) << (7 * k)
        if not c & 0x80:
            # reject non-minimal encodings
            if k > 0 and c == 0:
                return None
            return v, i + k + 1
    return None


def parse(payload: bytes):
    """-> dict(sig_cnt, sig_off, acct_off, msg_off, version) or None."""
    b = payload
    if len(b) > TXN_MTU:
        return None
    r = _cu16(b, 0)
    if r is None:
        return None
    sig_cnt, i = r
    if not 1 <= sig_cnt <= SIG_MAX:
        return None
    sig_off = i
    i += 64 * sig_cnt
    msg_off = i
    if i >= len(b):
        return None
    version = -1
    if b[i] & 0x80:
        version = b[i] & 0x7F
        if version != 0:
            return None
        i += 1
    if i + 3 > len(b):
        return None
    req, ro_signed, ro_unsigned = b[i], b[i + 1], b[i + 2]
    i += 3
    if req != sig_cnt or ro_signed >= req:
        return None
    r = _cu16(b, i)
    if r is None:
        return None
    acct_cnt, i = r
    if acct_cnt < req or acct_cnt > ACCT_ADDR_MAX or ro_unsigned > acct_cnt - req:
        return None
    acct_off = i
    i += 32 * acct_cnt + 32  # addresses + recent blockhash
    if i > len(b):
        return None
    r = _cu16(b, i)
    if r is None:
        return None
    instr_cnt, i = r
    for _ in range(instr_cnt):
        if i >= len(b):
            return None
        i += 1  # program id index
        for _ in range(2):  # accounts, data
            r = _cu16(b, i)
            if r is None:
                return None
            n, i = r
            i += n
            if i > len(b):
                return None
    if version == 0:
        r = _cu16(b, i)
        if r is None:
            return None
        lut_cnt, i = r
        for _ in range(lut_cnt):
            i += 32
            for _ in range(2):
                r = _cu16(b, i)
                if r is None:
                    return None
                n, i = r
                i += n
                if i > len(b):
                    return None
    if i != len(b):
        return None
    return {"sig_cnt": sig_cnt, "sig_off": sig_off, "acct_off": acct_off, "msg_off": msg_off, "version": version}


def descs_for(payload: bytes, base: int = 0):
    """Engine descriptors for one txn placed at blob offset `base`."""
    t = parse(payload)
    if t is None:
        return None
    d = np.zeros(t["sig_cnt"], DESC_DTYPE)
    for j in range(t["sig_cnt"]):
        d[j] = (base + t["sig_off"] + 64 * j, base + t["acct_off"] + 32 * j, base + t["msg_off"],
                len(payload) - t["msg_off"])
    return d
