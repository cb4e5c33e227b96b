"""Generates tests/golden/txn_parse_golden.json from the REFERENCE parser
(src/ballet/txn/fd_txn_parse.c compiled in place into
oracle/_ref/libfdref.so by oracle/Makefile): the descriptor of each
fixture, and for the test_mutate input set of each fixture
(src/ballet/txn/test_txn_parse.c:107-190) the sha256 over all results and
the final parse counters.  Run from the repo root:
    make -C oracle ref && python tests/golden/make_txn_golden.py"""
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from firedancer_amd import txn  # noqa: E402
from test_txn import _parser, fixtures, sweep  # noqa: E402


def main():
    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfdref.so"))
    fn = _parser(ref, "ref_txn_parse")
    out = {"source": "reference fd_txn_parse (oracle/_ref/libfdref.so)", "fixtures": [], "sweep": []}
    for p in fixtures():
        buf = ctypes.create_string_buffer(txn.TXN_MAX_SZ)
        fp = fn(p, len(p), buf, None)
        out["fixtures"].append({"footprint": fp, "raw": buf.raw[:fp].hex()})
        digest, ctr = sweep(fn, p)
        out["sweep"].append({"sha256": digest, "success_cnt": ctr[0], "failure_cnt": ctr[1], "failure_ring": ctr[2]})
    json.dump(out, open(os.path.join(ROOT, "tests", "golden", "txn_parse_golden.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
