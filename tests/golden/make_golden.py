#!/usr/bin/env python3
"""Regenerate the committed golden fixtures under tests/golden/.

Runs only in the build container (needs /root/reference and the
reference library oracle/_ref/libfdref.so built by oracle/Makefile).
Everything written is data -- inputs and expected outputs:

  malleability_should_{pass,fail}.bin  reference's own KAT files
      (src/ballet/ed25519/test_ed25519_signature_malleability_*.bin,
      196 + 200 (sig, pub) pairs over msg "Zcash"), copied byte-for-byte
  transaction{1,2,3}.bin                reference's txn fixtures
      (src/ballet/txn/fixtures/)
  sha512_vectors.json                   SHA-512 known answers: NIST CAVP
      ShortMsg (all 129), LongMsg (all 128, messages as hex), Monte seed +
      100 checkpoints (src/ballet/sha512/cavp/), and the 45 OpenSSL-derived
      vectors of src/ballet/sha512/fd_sha512_test_vector.c
  ed25519_vectors.json                  RFC 8032 TEST 1/2/3/1024/SHA(abc)
      (src/wiredancer/py/ref_ed25519.py:228-386) and the three Q2 limb-alias
      vectors of SURVEY.md section 8c, each with the reference's code
  corpus_*.npz                          packed corpora (blob, desc) with
      the reference library's per-signature codes (expected)
"""
import ctypes
import json
import os
import re
import shutil
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
REF = os.environ.get("FD_REFERENCE", "/root/reference")
sys.path.insert(0, ROOT)

from firedancer_amd import corpus  # noqa: E402


def ref_lib():
    L = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfdref.so"))
    L.ref_verify.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_void_p, ctypes.c_void_p]
    L.ref_verify.restype = ctypes.c_int
    return L


def ref_verify(L, msg, sig, pub):
    m = ctypes.create_string_buffer(bytes(msg), max(1, len(msg)))
    return L.ref_verify(m, len(msg), bytes(sig), bytes(pub))


def ref_batch(L, b):
    sig, pub, data, off, sz = b.flat()
    out = np.zeros(len(b), np.int32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    L.ref_verify_batch(ctypes.c_ulong(len(b)), P(sig), P(pub), P(data), P(off), P(sz), P(out), 8)
    return out


def copy_bins():
    src = os.path.join(REF, "src", "ballet", "ed25519")
    for k in ("pass", "fail"):
        shutil.copyfile(os.path.join(src, f"test_ed25519_signature_malleability_should_{k}.bin"),
                        os.path.join(HERE, f"malleability_should_{k}.bin"))
    for i in (1, 2, 3):
        shutil.copyfile(os.path.join(REF, "src", "ballet", "txn", "fixtures", f"transaction{i}.bin"),
                        os.path.join(HERE, f"transaction{i}.bin"))


def parse_rsp(path):
    recs, cur = [], {}
    for line in open(path):
        line = line.strip()
        m = re.match(r"^(\w+)\s*=\s*(\S*)$", line)
        if m:
            cur[m.group(1)] = m.group(2)
            if m.group(1) == "MD":
                recs.append(cur)
                cur = {}
    return recs


def parse_c_vectors(path):
    """{ "str" "str"..., <sz>UL, { _(xx),... } } entries of fd_sha512_test_vector.c"""
    txt = open(path).read()
    body = txt[txt.index("fd_sha512_test_vector[] = {"):]
    out = []
    for m in re.finditer(r'\{\s*((?:"(?:[^"\\]|\\.)*"\s*)+),\s*(\d+)UL,\s*\{([^}]*)\}\s*\}', body):
        s = "".join(re.findall(r'"((?:[^"\\]|\\.)*)"', m.group(1)))
        s = bytes(s, "latin1").decode("unicode_escape").encode("latin1")
        sz = int(m.group(2))
        h = bytes(int(x, 16) for x in re.findall(r"_\((\w\w)\)", m.group(3)))
        assert len(s) == sz and len(h) == 64
        out.append({"msg": s.hex(), "md": h.hex()})
    return out


def sha_vectors():
    cav = os.path.join(REF, "src", "ballet", "sha512", "cavp")
    short = [{"msg": r["Msg"] if int(r["Len"]) else "", "md": r["MD"]} for r in parse_rsp(os.path.join(cav, "SHA512ShortMsg.rsp"))]
    long_ = [{"msg": r["Msg"], "md": r["MD"]} for r in parse_rsp(os.path.join(cav, "SHA512LongMsg.rsp"))]
    mt = parse_rsp(os.path.join(cav, "SHA512Monte.rsp"))
    seed = re.search(r"Seed = (\w+)", open(os.path.join(cav, "SHA512Monte.rsp")).read()).group(1)
    monte = {"seed": seed, "md": [r["MD"] for r in mt]}
    fdv = parse_c_vectors(os.path.join(REF, "src", "ballet", "sha512", "fd_sha512_test_vector.c"))
    json.dump({"cavp_short": short, "cavp_long": long_, "cavp_monte": monte, "fd_test_vector": fdv},
              open(os.path.join(HERE, "sha512_vectors.json"), "w"))
    return len(short), len(long_), len(fdv)


Q2 = [
    ("5bba42a60de96030d8f6a85dc5809e3f39a210671f50ee0ffdab810e18725a49",
     "a53f00568d07e4944ee86da222b258beae6d8353024faf57de1fa83b05eea496267f66788337eab61e0d36da454c46700ad217fb3cb08d3d016548e4ff5be803",
     "562c7b301299d47deefe44c5368b77333c214b79b3e7dc03b091f0add168c0910740ac7544423faa742c3ba3d5286c624e1c5174ae4ccad097bea9f3c3cc197f33b0c640b71ae479e30fb2b7159bfb099c9780aa80fff0c1ea9682838b906f8677ea561bef530df8f714bea2b6eeb81b7b468ab64220d9d62a00a557e66bb35d"),
    ("a8c5f0b9a0cad87801e0e550c7b4cda39c96cc31b6de89123437e41c3f42ccfe",
     "588e6a12357767161aae6b35a7768481883861dcb399c0929ba2319214871d93895b3ab2404066f4e92dba7c688dbca7874ef5c16bedcb1efc6eb50560fe3602",
     "b594272285085ae80737ae28cf824783a8788d96d301ef3376d5f6de6599498fe92ab86784c593a3d42802cb97dcd15797351268f765787d68e4b6053cef065acc426921518d814afde0ca82fd788941a87e9468af2070c05755a2caeb6bdd34b8d108fe1ae96d59f8017eb0fe18c1a6da300403730cc3344d8cf5ecdba1bce9"),
    ("1935951cae485585719b256b1132ccbc729da20b718cfe2950c18dcdd82bbd71",
     "f064a139d45ec0994e332d79364ddd8c2894a3a9b97b571e864efe0cf2fbae0055b9ce729e97564fe0bf3444b29719f1908388a5ff1807355cff0a69561fb003",
     "fc2f6a47b996987a34e02bc58cc0e2f84144f1fa4a07d2964f2695e7daecdf8c1bb177623f9fe1d12b12a087383fa17153234d17507d1d45b5e009f968528efd7e51c1781977306ae975fee54e1665da6896fc2d53ce9ea9340282bbae55102db2dbaffb5798b0874037889b445e8b00afeeb1ad12f53e389f5cd7bc238bd4c9"),
]


def ed_vectors(L):
    txt = open(os.path.join(REF, "src", "wiredancer", "py", "ref_ed25519.py")).read()
    blocks = re.split(r"# -----TEST ", txt)[1:]
    vecs = []
    for blk in blocks:
        name = blk.split("\n", 1)[0].strip()
        def grab(var):
            return "".join(re.findall(var + r'\s*\+?=\s*bytes\.fromhex\("(\w*)"\)', blk))
        pub, msg, sig = grab("keyP"), grab("msg"), grab("sigt")
        if not pub or not sig:
            m = re.search(r"msg\s*=\s*b'([^']*)'", blk)
            continue
        if "msg  = b''" in blk or "msg = b''" in blk:
            msg = ""
        code = ref_verify(L, bytes.fromhex(msg), bytes.fromhex(sig), bytes.fromhex(pub))
        vecs.append({"name": "rfc8032_" + name, "pub": pub, "sig": sig, "msg": msg, "expected": code})
    for i, (pub, sig, msg) in enumerate(Q2):
        code = ref_verify(L, bytes.fromhex(msg), bytes.fromhex(sig), bytes.fromhex(pub))
        vecs.append({"name": f"q2_limb_alias_{i}", "pub": pub, "sig": sig, "msg": msg, "expected": code})
    json.dump(vecs, open(os.path.join(HERE, "ed25519_vectors.json"), "w"), indent=1)
    return vecs


def small_order_cross(seed=11):
    """Every small-order encoding as A, as R, and as both, over valid sigs."""
    encs = corpus.small_order_encodings()
    base = corpus.simple(3 * len(encs) + len(encs) ** 2, 64, seed=seed)
    blob = base.blob
    d = base.desc
    k = 0
    for e in encs:                      # as A
        o = int(d[k]["pub_off"]); blob[o:o + 32] = np.frombuffer(e, np.uint8); k += 1
    for e in encs:                      # as R
        o = int(d[k]["sig_off"]); blob[o:o + 32] = np.frombuffer(e, np.uint8); k += 1
    for e in encs:                      # as R with S = 0
        o = int(d[k]["sig_off"]); blob[o:o + 32] = np.frombuffer(e, np.uint8); blob[o + 32:o + 64] = 0; k += 1
    for ea in encs:                     # both
        for er in encs:
            o = int(d[k]["pub_off"]); blob[o:o + 32] = np.frombuffer(ea, np.uint8)
            o = int(d[k]["sig_off"]); blob[o:o + 32] = np.frombuffer(er, np.uint8)
            k += 1
    return corpus.Batch(blob, d, np.zeros(len(d), np.int8))


def save_corpus(L, name, b):
    exp = ref_batch(L, b)
    np.savez_compressed(os.path.join(HERE, f"corpus_{name}.npz"), blob=b.blob, desc=b.desc, label=b.label, expected=exp)
    vals, cnts = np.unique(exp, return_counts=True)
    print(name, len(b), dict(zip(vals.tolist(), cnts.tolist())))


def main():
    L = ref_lib()
    copy_bins()
    print("sha vectors", sha_vectors())
    print("ed vectors", [(v["name"], v["expected"]) for v in ed_vectors(L)])
    save_corpus(L, "adversarial", corpus.adversarial(6144, 128, seed=101, invalid_frac=0.25))
    save_corpus(L, "txn1232", corpus.solana_txns(768, seed=102))
    save_corpus(L, "small_order", small_order_cross())
    save_corpus(L, "msgsizes", corpus.concat([corpus.simple(16, sz, seed=200 + sz) for sz in
                                              (0, 1, 31, 32, 33, 47, 48, 63, 64, 111, 112, 127, 128, 129, 239, 240, 1023, 1232)]))


if __name__ == "__main__":
    main()
