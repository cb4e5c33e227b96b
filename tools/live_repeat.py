"""Repeat one live-harness configuration (tests/vt_live.cpp) N times and
stop at the first run that fails or outlives its limit: a hang shows the
harness's own report (tile batch state, engine slot states).

  python tools/live_repeat.py [--runs 4] [--staged 1] [--mode copy] [--tiles 2]

The corpus is the one tests/test_verify_tile_live.py::test_two_tiles_one_engine
uses (20,000 signatures, 1-12 per txn, ~10 % with a corrupted signature),
checked against the reference build (oracle/_ref)."""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--runs", type=int, default=4)
    ap.add_argument("--staged", type=int, default=1)
    ap.add_argument("--mode", default="copy")
    ap.add_argument("--tiles", type=int, default=2)
    ap.add_argument("--rate", type=float, default=10e6)
    ap.add_argument("--seconds", type=float, default=2)
    ap.add_argument("--limit", type=float, default=150)
    a = ap.parse_args()
    import ctypes
    import numpy as np
    from conftest import oracle_batch
    from live_common import quiet_cpus, write_frags
    import test_verify_tile_live as T
    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfdref.so"))
    frags, ok = T._cyclic_corpus(ref, 20000, 73)
    d = tempfile.mkdtemp()
    p, ex = os.path.join(d, "frags.bin"), os.path.join(d, "expect.bin")
    write_frags(p, frags)
    ok.astype(np.uint8).tofile(ex)
    spf = np.mean([f[((int.from_bytes(f[-2:], "little") + 1) & ~1) + 1] for f in frags])
    env = dict(os.environ)
    if a.staged:
        env["FD_VERIFY_TILE_COPY_STAGED"] = "1"
    for k in range(a.runs):
        c = quiet_cpus(2 * a.tiles)
        args = [T.EXE, p, f"mode={a.mode}", f"rate={a.rate / spf / a.tiles}", f"seconds={a.seconds}",
                f"tiles={a.tiles}", "share=1", "depth=16384", "batch=4096", "eng_depth=8", f"expect={ex}"]
        if c:
            args.append(f"cpus={c}")
        t0 = time.time()
        try:
            r = subprocess.run(args, capture_output=True, text=True, timeout=a.limit, env=env)
        except subprocess.TimeoutExpired as e:
            err = e.stderr.decode(errors="replace") if isinstance(e.stderr, bytes) else (e.stderr or "")
            print(json.dumps({"run": k, "timeout_s": a.limit, "stderr_tail": err[-3000:]}), flush=True)
            return 1
        lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
        rec = json.loads(lines[-1]) if lines else {"no_json": r.stdout[-1000:]}
        keep = {k2: rec.get(k2) for k2 in ("error", "tiles", "pub", "mismatch", "false_pub", "booted", "err", "lat", "diag")}
        print(json.dumps({"run": k, "rc": r.returncode, "s": round(time.time() - t0, 1), **keep,
                          "stderr_tail": r.stderr[-1500:] if r.returncode else ""}), flush=True)
        if r.returncode:
            return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
