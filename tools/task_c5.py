#!/usr/bin/env python3
"""C5 as a validator runs it: the verify tile TASK
(fd_verify_tile_task.run, its own run loop, its own wait bound) fed by a
live producer thread over a 16,384-frag mcache/dcache link shaped like the
reference's QUIC -> verify link (tests/vt_live.cpp), HALT only at the end.

For each offered load (verifies/s) and mode (copy / in place) it runs
--seconds of stream and records, one JSON line per point:
  - offered and achieved rates (frags and signatures taken per second);
  - tsorig (the producer's write) -> tspub (the tile's publish), p50 / p99 /
    p99.9 / max, the first --warm seconds excluded;
  - the reference check over EVERY publish of the run: the corpus (1..12
    signatures per txn, ~10% with a corrupted signature, all distinct) is
    verified by the reference's own fd_ed25519_verify (oracle/_ref/
    libfdref.so) up front; each publish must be a frag the reference
    publishes (false_pub), carry exactly the bytes written for its seq
    (mismatch) and come in seq order; with no overrun the publish count
    must equal the reference-passing frags taken (pub == taken_pass_expected);
  - the tile's counters (OVRN_CNT: frags the producer lapped before their
    publish, in place; AGE_CNT: batches closed by the wait bound).

usage: tools/task_c5.py --rates 1e6,10e6,30e6,45e6 --modes copy,inplace --seconds 60 --out profiles/r06_task_c5_60s.jsonl
"""
import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def corpus(n_sigs, seed):
    from firedancer_amd import corpus as C, txn
    b = C.solana_txns(n_sigs, seed=seed, sig_dist=[1 / 12] * 12, nthreads=16)
    starts = sorted({int(d["sig_off"]) // C.TXN_MTU * C.TXN_MTU for d in b.desc})
    pay = [bytearray(b.blob[s:s + C.TXN_MTU]) for s in starts]
    rng = np.random.default_rng(seed)
    for q in pay:
        if rng.random() < 0.10:
            j = int(rng.integers(0, q[0]))
            q[1 + 64 * j + int(rng.integers(8, 64))] ^= 1 << int(rng.integers(0, 8))
    return [txn.frag(bytes(q)) for q in pay]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rates", default="1e6,10e6,30e6,45e6", help="offered verifies/s, comma-separated")
    ap.add_argument("--modes", default="copy,inplace")
    ap.add_argument("--seconds", type=float, default=60.0)
    ap.add_argument("--warm", type=float, default=2.0)
    ap.add_argument("--sigs", type=int, default=53248, help="signatures in the corpus (cycled)")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--eng-depth", type=int, default=8)
    ap.add_argument("--depth", type=int, default=16384, help="mcache/dcache frags (default.toml receive_buffer_size)")
    ap.add_argument("--max-wait-ns", type=int, default=0)
    ap.add_argument("--tiles", type=int, default=1, help="verify tiles on the GPU, each with its own link and producer")
    ap.add_argument("--share", type=int, default=0, help="1: the tiles share one engine (fd_verify_tile_args_t.shared_gpu)")
    ap.add_argument("--rt", type=int, default=0, help="1: the harness's spinning threads ask for SCHED_FIFO (reported as rt_threads)")
    ap.add_argument("--sample", type=int, default=0, help="1: sample where tile 0's thread waits (tile0_syscall_samples)")
    ap.add_argument("--copy-staged", type=int, default=0,
                    help="1: copying tiles build batches in the engine's staged slots ($FD_VERIFY_TILE_COPY_STAGED)")
    ap.add_argument("--l3-pairs", type=int, default=1,
                    help="1: producer k and tile k on cores sharing a last-level cache (fa.quiet_cpus pairs)")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    import ctypes
    from conftest import oracle_batch
    from live_common import expected_cyclic, run, write_frags
    import firedancer_amd as fa
    ref = ctypes.CDLL(os.path.join(ROOT, "oracle", "_ref", "libfdref.so"))
    frags = corpus(a.sigs, 606)
    ok = expected_cyclic(frags, ref, oracle_batch)
    spf = float(np.mean([fa_sigs(f) for f in frags]))
    tmp = tempfile.mkdtemp()
    fp, ex = os.path.join(tmp, "frags.bin"), os.path.join(tmp, "expect.bin")
    write_frags(fp, frags)
    ok.astype(np.uint8).tofile(ex)
    from live_common import quiet_cpus
    pin = quiet_cpus(2 * a.tiles, pairs=bool(a.l3_pairs))   # producer k, tile k: the quietest cores of the GPU's NUMA node
    exe = os.path.join(ROOT, "firedancer_amd", "vt_live")
    out = open(a.out, "a") if a.out else None
    # ',' or '+' between values ('+' survives tools/gpu.sh's py= step)
    for mode in a.modes.replace("+", ",").split(","):
        for r in [float(x) for x in a.rates.replace("+", ",").split(",")]:
            kw = dict(mode=mode, rate=r / spf / a.tiles, tiles=a.tiles, share=a.share, seconds=a.seconds, warm=a.warm, depth=a.depth, batch=a.batch,
                      eng_depth=a.eng_depth, max_wait_ns=a.max_wait_ns, expect=ex, rt=a.rt, sample=a.sample)
            if pin:
                kw["cpus"] = pin
            t0 = time.time()
            env = dict(os.environ, FD_VERIFY_TILE_COPY_STAGED="1") if a.copy_staged else None
            d = run(exe, fp, timeout=a.seconds + 120, env=env, **kw)
            if "error" in d:      # the harness refused the configuration (e.g. an engine depth past the maximum)
                print(json.dumps({"error": d["error"], "config": kw, "rc": d["rc"]}), flush=True)
                continue
            d.pop("stderr", None)
            if mode == "copy":
                d["copy_buffers"] = "engine staged slots" if a.copy_staged else "tile's own registered buffers"
            d["l3_pairs"] = bool(a.l3_pairs)
            d.update({
                      "offered_verifies_s": r, "sigs_per_frag": spf, "corpus_frags": len(frags),
                      "corpus_reference_pass": int(ok.sum()), "cpus": pin, "wall_s": time.time() - t0,
                      "kernels_id": fa.kernels_id(),
                      "reference_check": {"publishes_checked": d["pub"], "false_pub": d["false_pub"],
                                          "byte_mismatch": d["mismatch"], "order_err": d["order_err"],
                                          "pub_equals_reference_set": d["pub"] == d["taken_pass_expected"]
                                          and d["diag"]["OVRN_CNT"] == 0 and d["ovrnp"] == 0 and d["ovrnr"] == 0,
                                          # with overruns: the reference's set of the frags taken, less
                                          # those the tile's overrun check dropped (tests/vt_live.cpp)
                                          "overrun_dropped": d["flagged"], "flagged_published": d["flag_pub"],
                                          "pub_equals_reference_set_less_overrun": d["pub"] == d["pub_expected_exact"]
                                          and d["flag_pub"] == 0}})
            line = json.dumps(d)
            print(line, flush=True)
            if out:
                out.write(line + "\n")
                out.flush()


def fa_sigs(f):
    psz = int.from_bytes(f[-2:], "little")
    return f[((psz + 1) & ~1) + 1]


if __name__ == "__main__":
    main()
