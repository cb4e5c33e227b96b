"""Synthetic corpora for the sigverify path.

All corpora are packed batches: one uint8 blob plus one
``DESC_DTYPE`` descriptor per signature (offsets of R||S, public key and
message inside the blob), the engine's input format.

  C1  random 128-byte messages, all valid               (solana=False)
  C2  Solana-MTU legacy txns of exactly 1232 bytes with 1 or 2
      signatures (p = 0.7 / 0.3); msg = payload[1+64k:]  (solana_txns)
  C3  adversarial mix (adversarial): flips, S >= L, the early-accept S
      pattern, non-canonical and small-order encodings, points off the
      curve, mixed-order keys
  C4  one shared message, many signers                   (single_msg)

Keys come from deterministic per-index seeds, signatures from the
product's host signer (fd_ed25519_sign_batch); no test oracle is used
here, so bench.py can build its workload on the GPU box.
"""
from __future__ import annotations

import numpy as np

from . import DESC_DTYPE, sign_batch, lib, _p

P = 2**255 - 19
L = 2**252 + 27742317777372353535851937790883648493
D = (-121665 * pow(121666, P - 2, P)) % P
SQRTM1 = pow(2, (P - 1) // 4, P)
TXN_MTU = 1232  # FD_TPU_MTU, src/ballet/fd_ballet_base.h:9


# ---------------------------------------------------------------- math helpers
def _inv(x):
    return pow(x, P - 2, P)


def _xrecover(y, sign):
    """x for y (mod p) with the given sign, or None if not on the curve."""
    y %= P
    u, v = (y * y - 1) % P, (D * y * y + 1) % P
    x = pow(u * pow(v, 3, P) * pow(u * pow(v, 7, P), (P - 5) // 8, P), 1, P)
    if (v * x * x - u) % P != 0:
        if (v * x * x + u) % P != 0:
            return None
        x = x * SQRTM1 % P
    if x % 2 != sign:
        x = (P - x) % P
    return x


def _add(p1, p2):
    x1, y1 = p1
    x2, y2 = p2
    t = D * x1 * x2 * y1 * y2
    return ((x1 * y2 + x2 * y1) * _inv(1 + t) % P, (y1 * y2 + x1 * x2) * _inv(1 - t) % P)


def _mul(k, pt):
    r, q = (0, 1), pt
    while k:
        if k & 1:
            r = _add(r, q)
        q = _add(q, q)
        k >>= 1
    return r


def _enc(pt, y_override=None):
    x, y = pt
    y = y if y_override is None else y_override
    b = bytearray(y.to_bytes(32, "little"))
    b[31] |= (x & 1) << 7
    return bytes(b)


def _dec(b):
    y = int.from_bytes(b, "little") & ((1 << 255) - 1)
    x = _xrecover(y, b[31] >> 7)
    return None if x is None else (x, y % P)


BASE = (_xrecover(4 * _inv(5) % P, 0), 4 * _inv(5) % P)


def torsion_points():
    """The 8 points of order dividing 8."""
    # an order-8 point: y^2 solves the torsion equation; find by scanning the
    # order-4/8 structure: take any point Q, then [L]Q has order | 8.
    pts = set()
    y = 2
    while len(pts) < 8:
        x = _xrecover(y, 0)
        if x is not None:
            t = _mul(L, (x, y))
            q = t
            for _ in range(8):
                pts.add(q)
                q = _add(q, t)
        y += 1
    return sorted(pts)


def small_order_encodings():
    """All 14 encodings of small-order points accepted by lax decoding:
    5 distinct y values (identity, order 2, order 4 (y=0), order 8 pair)
    x 2 sign bits, plus non-canonical y+p for y in {0, 1} x 2 signs.
    (x = 0 points keep both sign bits: the lax decoder accepts
    'negative zero')"""
    ys = sorted({pt[1] for pt in torsion_points()})
    encs = []
    for y in ys:
        for s in (0, 1):
            b = bytearray(y.to_bytes(32, "little"))
            b[31] |= s << 7
            encs.append(bytes(b))
    for y in (0, 1):
        for s in (0, 1):
            b = bytearray((y + P).to_bytes(32, "little"))
            b[31] |= s << 7
            encs.append(bytes(b))
    return encs


def off_curve_encodings(n, rng):
    out = []
    while len(out) < n:
        y = int.from_bytes(rng.bytes(32), "little") & ((1 << 255) - 1)
        if y < P and _xrecover(y, 0) is None:
            out.append(bytes(bytearray(y.to_bytes(32, "little"))))
    return out


# ---------------------------------------------------------------- packing
class Batch:
    """A packed batch plus per-signature metadata."""

    def __init__(self, blob, desc, label=None):
        self.blob = np.ascontiguousarray(blob, dtype=np.uint8)
        self.desc = np.ascontiguousarray(desc, dtype=DESC_DTYPE)
        self.label = label

    def __len__(self):
        return len(self.desc)

    def sig(self, i):
        o = int(self.desc[i]["sig_off"])
        return bytes(self.blob[o:o + 64])

    def pub(self, i):
        o = int(self.desc[i]["pub_off"])
        return bytes(self.blob[o:o + 32])

    def msg(self, i):
        o, s = int(self.desc[i]["msg_off"]), int(self.desc[i]["msg_sz"])
        return bytes(self.blob[o:o + s])

    def flat(self):
        """SoA arrays (sig[n,64], pub[n,32], data, msg_off[u64], msg_sz[u32]) for CPU checkers."""
        n = len(self)
        so = self.desc["sig_off"].astype(np.int64)
        po = self.desc["pub_off"].astype(np.int64)
        sig = self.blob[so[:, None] + np.arange(64)[None, :]] if n else np.zeros((0, 64), np.uint8)
        pub = self.blob[po[:, None] + np.arange(32)[None, :]] if n else np.zeros((0, 32), np.uint8)
        return (np.ascontiguousarray(sig), np.ascontiguousarray(pub), self.blob,
                self.desc["msg_off"].astype(np.uint64), self.desc["msg_sz"].astype(np.uint32))

    def tile(self, reps):
        """Repeat the descriptors (not the blob): same bytes, reps x the signatures."""
        return Batch(self.blob, np.tile(self.desc, reps), None if self.label is None else np.tile(self.label, reps))


def _seeds(n, seed):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, (n, 32), dtype=np.uint8), rng


def simple(n, msg_sz=128, seed=0, nthreads=8):
    """C1: n x (msg_sz random bytes, key i from seed stream), all valid.
    Blob layout per item: R||S (64) | pub (32) | msg."""
    seeds, rng = _seeds(n, seed)
    stride = 96 + msg_sz
    blob = np.zeros(n * stride + 64, np.uint8)
    base = np.arange(n, dtype=np.int64) * stride
    msgs = rng.integers(0, 256, (n, msg_sz), dtype=np.uint8)
    for k in range(msg_sz):
        blob[base + 96 + k] = msgs[:, k]
    off = (base + 96).astype(np.uint64)
    sz = np.full(n, msg_sz, np.uint32)
    pub, sig = sign_batch(seeds, blob, off, sz, nthreads)
    for k in range(64):
        blob[base + k] = sig[:, k]
    for k in range(32):
        blob[base + 64 + k] = pub[:, k]
    desc = np.zeros(n, DESC_DTYPE)
    desc["sig_off"], desc["pub_off"], desc["msg_off"], desc["msg_sz"] = base, base + 64, base + 96, msg_sz
    return Batch(blob, desc, np.zeros(n, np.int8))


def solana_txns(n_sigs, seed=0, p2=0.3, max_sigs_per_txn=2, nthreads=8, sig_dist=None):
    """C2/C5: legacy Solana txns of exactly TXN_MTU bytes.

    payload = compact_u16(k) | k x sig | message, message =
      header(3) | compact_u16(k+1) | k signer keys + 1 program key |
      blockhash(32) | compact_u16(1) | one instruction whose data fills the
      MTU (up to 12 signatures fit).  Every txn parses with fd_txn_parse.
    Signature j covers message = payload[1+64k:] with account key j.
    sig count: 1 or 2 with p(2)=p2, or drawn from sig_dist (list of
    probabilities for k = 1..len)."""
    rng = np.random.default_rng(seed)
    ks = []
    tot = 0
    while tot < n_sigs:
        if sig_dist is not None:
            k = int(rng.choice(np.arange(1, len(sig_dist) + 1), p=sig_dist))
        else:
            k = 2 if rng.random() < p2 else 1
        k = min(k, n_sigs - tot)
        ks.append(k)
        tot += k
    ntx = len(ks)
    blob = np.zeros(ntx * TXN_MTU + 64, np.uint8)
    desc = np.zeros(n_sigs, DESC_DTYPE)
    seeds = rng.integers(0, 256, (n_sigs, 32), dtype=np.uint8)
    pubs = np.zeros((n_sigs, 32), np.uint8)
    lib().fd_ed25519_public_batch(n_sigs, _p(seeds), _p(pubs), nthreads)
    s = 0
    msg_off = np.zeros(n_sigs, np.uint64)
    msg_sz = np.zeros(n_sigs, np.uint32)
    filler = rng.integers(0, 256, TXN_MTU, dtype=np.uint8)
    for t, k in enumerate(ks):
        b = t * TXN_MTU
        m = k + 1  # signers + the (readonly, unsigned) program account
        mo = b + 1 + 64 * k
        blob[b] = k
        blob[mo:mo + 3] = (k, 0, 1)
        blob[mo + 3] = m
        for j in range(k):
            blob[mo + 4 + 32 * j: mo + 4 + 32 * (j + 1)] = pubs[s + j]
        rest = mo + 4 + 32 * m                  # after the account keys
        blob[mo + 4 + 32 * k:rest] = filler[:32 * (m - k)]
        blob[rest:rest + 32] = filler[32:64]    # recent blockhash, unique per txn
        blob[rest:rest + 8] = np.frombuffer(np.uint64(t).tobytes(), np.uint8)
        blob[rest + 8:rest + 16] = np.frombuffer(np.uint64(seed).tobytes(), np.uint8)
        rest += 32
        room = b + TXN_MTU - (rest + 3)         # instr count, program id, account count
        dl = room - 1 if room - 1 < 128 else room - 2
        blob[rest] = 1                          # one instruction
        blob[rest + 1] = m - 1                  # program id index
        blob[rest + 2] = 0                      # no account indices
        if dl < 128:                            # minimal compact-u16 data length
            blob[rest + 3] = dl
            d0 = rest + 4
        else:
            blob[rest + 3] = 0x80 | (dl & 0x7F)
            blob[rest + 4] = dl >> 7
            d0 = rest + 5
        blob[d0:b + TXN_MTU] = filler[:dl]
        for j in range(k):
            desc[s + j] = (b + 1 + 64 * j, mo + 4 + 32 * j, mo, TXN_MTU - 1 - 64 * k)
            msg_off[s + j] = mo
            msg_sz[s + j] = TXN_MTU - 1 - 64 * k
        s += k
    sig = np.zeros((n_sigs, 64), np.uint8)
    lib().fd_ed25519_sign_batch(n_sigs, _p(seeds), _p(blob), _p(msg_off), _p(msg_sz), _p(pubs), _p(sig), -nthreads)
    so = desc["sig_off"].astype(np.int64)
    for c in range(64):
        blob[so + c] = sig[:, c]
    return Batch(blob, desc, np.zeros(n_sigs, np.int8))


def single_msg(n, msg_sz=256, seed=0, nthreads=8):
    """C4: one shared message (vote-txn shaped), n signers."""
    seeds, rng = _seeds(n, seed)
    msg = rng.integers(0, 256, msg_sz, dtype=np.uint8)
    blob = np.zeros(msg_sz + 96 * n + 64, np.uint8)
    blob[:msg_sz] = msg
    off = np.zeros(n, np.uint64)
    sz = np.full(n, msg_sz, np.uint32)
    pub, sig = sign_batch(seeds, blob, off, sz, nthreads)
    base = msg_sz + 96 * np.arange(n, dtype=np.int64)
    for k in range(64):
        blob[base + k] = sig[:, k]
    for k in range(32):
        blob[base + 64 + k] = pub[:, k]
    desc = np.zeros(n, DESC_DTYPE)
    desc["sig_off"], desc["pub_off"], desc["msg_off"], desc["msg_sz"] = base, base + 64, 0, msg_sz
    return Batch(blob, desc, np.zeros(n, np.int8)), msg, sig, pub


# ---------------------------------------------------------------- adversarial
# The three SURVEY.md section 8c (Q2) vectors as (msg, sig, pub) hex: valid
# signatures that the reference's AVX2 build rejects (ERR_MSG) through its
# limb compare of non-canonical coordinates (fd_ed25519_user.c:419-427).
Q2_VECTORS = [
    ("562c7b301299d47deefe44c5368b77333c214b79b3e7dc03b091f0add168c0910740ac7544423faa742c3ba3d5286c624e1c5174ae4ccad097bea9f3c3cc197f33b0c640b71ae479e30fb2b7159bfb099c9780aa80fff0c1ea9682838b906f8677ea561bef530df8f714bea2b6eeb81b7b468ab64220d9d62a00a557e66bb35d",
     "a53f00568d07e4944ee86da222b258beae6d8353024faf57de1fa83b05eea496267f66788337eab61e0d36da454c46700ad217fb3cb08d3d016548e4ff5be803",
     "5bba42a60de96030d8f6a85dc5809e3f39a210671f50ee0ffdab810e18725a49"),
    ("b594272285085ae80737ae28cf824783a8788d96d301ef3376d5f6de6599498fe92ab86784c593a3d42802cb97dcd15797351268f765787d68e4b6053cef065acc426921518d814afde0ca82fd788941a87e9468af2070c05755a2caeb6bdd34b8d108fe1ae96d59f8017eb0fe18c1a6da300403730cc3344d8cf5ecdba1bce9",
     "588e6a12357767161aae6b35a7768481883861dcb399c0929ba2319214871d93895b3ab2404066f4e92dba7c688dbca7874ef5c16bedcb1efc6eb50560fe3602",
     "a8c5f0b9a0cad87801e0e550c7b4cda39c96cc31b6de89123437e41c3f42ccfe"),
    ("fc2f6a47b996987a34e02bc58cc0e2f84144f1fa4a07d2964f2695e7daecdf8c1bb177623f9fe1d12b12a087383fa17153234d17507d1d45b5e009f968528efd7e51c1781977306ae975fee54e1665da6896fc2d53ce9ea9340282bbae55102db2dbaffb5798b0874037889b445e8b00afeeb1ad12f53e389f5cd7bc238bd4c9",
     "f064a139d45ec0994e332d79364ddd8c2894a3a9b97b571e864efe0cf2fbae0055b9ce729e97564fe0bf3444b29719f1908388a5ff1807355cff0a69561fb003",
     "1935951cae485585719b256b1132ccbc729da20b718cfe2950c18dcdd82bbd71")]

CASES = [
    "valid", "flip_R", "flip_S", "flip_msg", "flip_pub", "S_eq_L", "S_eq_L1", "S_top_big",
    "S_q1_early_accept", "noncanon_A", "noncanon_R", "small_A", "small_R", "small_both",
    "offcurve_A", "offcurve_R", "mixed_order_A", "negzero_A", "negzero_R",
]


def adversarial(n, msg_sz=128, seed=0, invalid_frac=0.1, nthreads=8):
    """C3: (1-invalid_frac) valid signatures, the rest split evenly over the
    invalid cases above.  Returns a Batch whose .label holds the case index."""
    return corrupt(simple(n, msg_sz, seed, nthreads), seed + 7919, invalid_frac)


def adversarial_txns(n, seed=0, invalid_frac=0.1, nthreads=8, **kw):
    """C3 at C2 shape: Solana-MTU txns (solana_txns; msg 1167 / 1103 B) with
    invalid_frac of the signatures corrupted over all the cases above.  In a
    txn the signer keys are part of the signed message, so a case that
    rewrites a key also changes its co-signers' message (the reference
    decides every code; the label names only what was done)."""
    return corrupt(solana_txns(n, seed=seed, nthreads=nthreads, **kw), seed + 7919, invalid_frac)


def corrupt(base, seed, invalid_frac=0.1, cases=None):
    """Corrupt invalid_frac of base's signatures in place, split evenly over
    CASES[1:] (or the named subset `cases`); .label receives the case index."""
    n = len(base)
    pick = [CASES.index(c) for c in cases] if cases else list(range(1, len(CASES)))
    rng = np.random.default_rng(seed)
    blob = base.blob
    desc = base.desc
    label = np.zeros(n, np.int8)
    n_bad = int(n * invalid_frac)
    idx = rng.choice(n, n_bad, replace=False)
    smalls = small_order_encodings()
    offc = off_curve_encodings(64, rng)
    torsion = [pt for pt in torsion_points() if pt != (0, 1)]
    for j, i in enumerate(idx):
        case = pick[j % len(pick)]
        label[i] = case
        name = CASES[case]
        so, po, mo, ms = (int(desc[i][f]) for f in ("sig_off", "pub_off", "msg_off", "msg_sz"))
        if name == "flip_R":
            blob[so + rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
        elif name == "flip_S":
            blob[so + 32 + rng.integers(0, 31)] ^= np.uint8(1 << rng.integers(0, 8))
        elif name == "flip_msg":
            if ms:
                blob[mo + rng.integers(0, ms)] ^= np.uint8(1 << rng.integers(0, 8))
        elif name == "flip_pub":
            blob[po + rng.integers(0, 32)] ^= np.uint8(1 << rng.integers(0, 8))
        elif name == "S_eq_L":
            blob[so + 32:so + 64] = np.frombuffer(L.to_bytes(32, "little"), np.uint8)
        elif name == "S_eq_L1":
            blob[so + 32:so + 64] = np.frombuffer((L + 1).to_bytes(32, "little"), np.uint8)
        elif name == "S_top_big":
            blob[so + 63] = rng.integers(0x11, 0x100)
        elif name == "S_q1_early_accept":
            blob[so + 63] = 0x10
            blob[so + 48:so + 63] = rng.integers(0, 256, 15, dtype=np.uint8)
            blob[so + 48 + rng.integers(0, 15)] |= np.uint8(1)
        elif name in ("noncanon_A", "noncanon_R"):
            y = int(rng.integers(0, 19))
            enc = bytearray((y + P).to_bytes(32, "little"))
            enc[31] |= int(rng.integers(0, 2)) << 7
            o = po if name == "noncanon_A" else so
            blob[o:o + 32] = np.frombuffer(bytes(enc), np.uint8)
        elif name in ("small_A", "small_R", "small_both"):
            e = smalls[int(rng.integers(0, len(smalls)))]
            if name in ("small_A", "small_both"):
                blob[po:po + 32] = np.frombuffer(e, np.uint8)
            if name in ("small_R", "small_both"):
                e2 = smalls[int(rng.integers(0, len(smalls)))]
                blob[so:so + 32] = np.frombuffer(e2, np.uint8)
        elif name == "offcurve_A":
            blob[po:po + 32] = np.frombuffer(offc[int(rng.integers(0, len(offc)))], np.uint8)
        elif name == "offcurve_R":
            blob[so:so + 32] = np.frombuffer(offc[int(rng.integers(0, len(offc)))], np.uint8)
        elif name == "mixed_order_A":
            a = _dec(bytes(blob[po:po + 32]))
            if a is not None:
                t = torsion[int(rng.integers(0, len(torsion)))]
                blob[po:po + 32] = np.frombuffer(_enc(_add(a, t)), np.uint8)
        elif name in ("negzero_A", "negzero_R"):
            # x = 0 points (y = 1 or p-1) with the sign bit set
            y = 1 if rng.integers(0, 2) else P - 1
            enc = bytearray(y.to_bytes(32, "little"))
            enc[31] |= 0x80
            o = po if name == "negzero_A" else so
            blob[o:o + 32] = np.frombuffer(bytes(enc), np.uint8)
    return Batch(blob, desc, label)


def concat(batches):
    """Concatenate packed batches into one (offsets rebased)."""
    blobs, descs, labels = [], [], []
    off = 0
    for b in batches:
        blen = len(b.blob)
        d = b.desc.copy()
        for f in ("sig_off", "pub_off", "msg_off"):
            d[f] = d[f] + off
        blobs.append(b.blob)
        descs.append(d)
        labels.append(b.label if b.label is not None else np.zeros(len(b), np.int8))
        off += blen
    return Batch(np.concatenate(blobs), np.concatenate(descs), np.concatenate(labels))


def from_triples(triples):
    """Batch from (msg, sig, pub) byte strings."""
    parts = []
    desc = np.zeros(len(triples), DESC_DTYPE)
    off = 0
    for i, (m, s, p) in enumerate(triples):
        desc[i] = (off, off + 64, off + 96, len(m))
        parts.append(bytes(s) + bytes(p) + bytes(m))
        off += 96 + len(m)
    blob = np.frombuffer(b"".join(parts) + b"\0" * 64, np.uint8).copy()
    return Batch(blob, desc, np.zeros(len(triples), np.int8))


def c3_windows(nwin, batch_sigs, seed, extra=None, extra_at=None, invalid_frac=0.1, nthreads=8):
    """The C2 ring's corpus with the C3 mix (BASELINE configs[1] batches,
    configs[2] content): nwin windows of batch_sigs signatures, each window
    contiguous in the blob (so a ring batch moves one ~4 MB span), drawn
    from adversarial_txns (invalid_frac corrupted over every case of CASES),
    plus the (msg, sig, pub) triples `extra` (e.g. the SURVEY Q2 vectors,
    which only the limb-exact path rejects) placed at the same offsets
    `extra_at` of every window.  Window w is desc[w*batch_sigs:(w+1)*batch_sigs]."""
    extra = list(extra or [])
    extra_at = list(extra_at if extra_at is not None else [(j + 1) * batch_sigs // (len(extra) + 1) for j in range(len(extra))])
    assert len(extra_at) == len(extra) and len(set(extra_at)) == len(extra_at) and all(0 <= a < batch_sigs for a in extra_at)
    k = batch_sigs - len(extra)
    adv = adversarial_txns(nwin * k, seed=seed, invalid_frac=invalid_frac, nthreads=nthreads)
    q = from_triples(extra) if extra else None
    parts = []
    for w in range(nwin):
        d = adv.desc[w * k:(w + 1) * k].copy()
        lo = int(min(d["sig_off"].min(), d["pub_off"].min(), d["msg_off"].min()))
        hi = int(max((d["sig_off"].astype(np.int64) + 64).max(), (d["pub_off"].astype(np.int64) + 32).max(),
                     (d["msg_off"].astype(np.int64) + d["msg_sz"]).max()))
        for f in ("sig_off", "pub_off", "msg_off"):
            d[f] = d[f] - lo
        parts.append(Batch(np.concatenate([adv.blob[lo:hi], np.zeros(64, np.uint8)]), d, adv.label[w * k:(w + 1) * k]))
        if q is not None:
            parts.append(q)
    b = concat(parts)
    if extra:
        # within each window: the extras (at k..batch_sigs) move to extra_at
        perm = np.empty(batch_sigs, np.int64)
        rest = [i for i in range(batch_sigs) if i not in set(extra_at)]
        perm[rest] = np.arange(k)
        perm[extra_at] = k + np.arange(len(extra))
        full = (np.arange(nwin)[:, None] * batch_sigs + perm[None, :]).ravel()
        b = Batch(b.blob, b.desc[full], b.label[full])
    return b



def c5_check_edits(frags):
    """The C5 check window's adversarial edits (tools/bench_tile.py
    --check-window, tests/test_c5_record.py), deterministic by index: frag i
    with i % 97 == 3 gets one bit of its first signature's R flipped
    (rejected by the verify), i % 89 == 5 repeats frag i - 1 (a dedup hit
    when that one was not itself rejected), i % 211 == 7 declares a 3-byte
    payload (does not parse)."""
    import struct
    out = list(frags)
    for i, f in enumerate(out):
        if i % 97 == 3:
            b = bytearray(f)
            b[1 + 10] ^= 0x04
            out[i] = bytes(b)
        elif i % 89 == 5 and i:
            out[i] = out[i - 1]
        elif i % 211 == 7:
            out[i] = f[:-2] + struct.pack("<H", 3)
    return out
