#!/usr/bin/env python3
"""bench.py -- Ed25519 batch verification throughput on MI355X.

Workload (BASELINE.json configs[1], "C2"): 4096-signature batches of
Solana-MTU (1232-byte) legacy txn payloads with 1-2 signatures per txn
(p = 0.7 / 0.3), all valid, synthetic (keys and messages from fixed
seeds, signed by the product's host signer).  One step = one pass of the
verify path over STEP_BATCHES such batches resident in HBM (one engine
launch: prep -> decomp -> dsm).  value = signatures verified by all ranks
/ max over ranks of the timed wall time (inputs already in HBM).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py
--gpus N): one process per GPU, each an independent replica on its own
shard of signatures (no data-path collective -- nothing is reduced);
RCCL only carries the timing barrier and the max-over-ranks.

Extra measurements on rank 0 at N=1:
  roofline     per-kernel HIP-event durations over the timed launches,
               algorithmic int32 ops / duration
  latency      C2 at its own granularity: 4096-signature batches of a
               C3-mix ring corpus (10 % invalid + the Q2 vectors in every
               batch) streamed through the per-GPU feeder and the engine's
               pinned ring (PCIe both ways included): closed loop (6 -- the
               main point --, 5, 7, 8 outstanding on a depth-8 ring, depth
               4, depth 1; push -> codes-on-host p50/p99), and an open-loop
               sweep of offered loads (25-40 M verifies/s) whose latency is
               scheduled arrival -> codes on the host; the headline is the
               highest offered load sustained at sched -> done p99 <= 1 ms.
               Every code of every leg is compared with the reference's.
  cpu_baseline the reference's own fd_ed25519_verify (oracle/_ref build,
               'reference') or the CPU restatement ('port') on a bounded
               sample of the same corpus, all host threads of this rank
"""
import argparse
import json
import math
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

BATCH_SIGS = 4096
STEP_BATCHES = 256
UNIQUE_SIGS = 65536

# ---- algorithmic work model --------------------------
# The path is bound by integer VALU issue.  Work is counted as the REFERENCE
# algorithm's operations (its field multiplies and squarings, SHA-512 blocks)
# priced at their minimal gfx950 issue cost in full-rate int32 lane-op slots:
#   a 32x32->64 multiply-accumulate (v_mad_i64_i32) issues at half rate = 2
#   slots (profiles/ubench_int_r01.txt: 0.43-0.45 of the v_add_u32 rate),
#   a 64-bit add/shift = 2 slots, a 32-bit op = 1 slot.
# fe_mul (FE_AVX_INL_MUL, avx/fd_ed25519_fe_avx_inl.h:484-590): 100 MACs
#   (200) + 15 operand pre-scales + 12 carries x (round 2 + shift 2 + add 2 +
#   sext 1) = 299.  fe_sq (FE_AVX_INL_SQN, :592-677): 55 MACs (110) + 30
#   pre-scales + 84 = 224; sq2 doubles 10 column sums (+20) = 244.
# SHA-512 block: 80 rounds x 40 + 64-word schedule x 26 + 16 = 4,900
#   (64-bit ops as 32-bit pairs).
SLOT_MUL, SLOT_SQ, SLOT_SQ2 = 299, 224, 244
SLOT_SHA_BLOCK = 4900
# per-verify reference op counts (251.5 doublings and
# 84.9 additions per verify, measured on the reference's slide statistics)
N_DBL, N_ADD = 251.5, 84.9
# DSM, split as the engine runs it (avx/fd_ed25519_ge.c:423-523,
#   fd_ed25519_user.c:419-427):
#   fd_k_dsm_setup: Ai table, 92 mul + 3 sq + 1 sq2 + 8 x 30 mix ops;
#   fd_k_dsm_pool:  each doubling SQN(1,1,1,2) + the p1p1->p2 conversion's 3
#                   MULs (X, Y, Z: the reference's 4-lane MUL leaves its 4th
#                   lane idle, avx/fd_ed25519_ge.c:521-522; the kernel issues
#                   3, fd_pool_dbl), each addition the 4-lane p3 conversion
#                   MUL + the 4-lane op MUL = 8 MULs, lane mixes DBL_MIX+X+Y
#                   50, SUBADD_12+SUB_MIX 70 int32 ops (3,140
#                   field ops per verify counts the conversion as 3);
#   fd_k_dsm_final: p2 conversion 3 mul + compare 2 mul.
SLOTS_DSM_SETUP = 92 * SLOT_MUL + 3 * SLOT_SQ + SLOT_SQ2 + 240
SLOTS_DSM_LOOP = ((3 * N_DBL + 8 * N_ADD) * SLOT_MUL + 3 * N_DBL * SLOT_SQ + N_DBL * SLOT_SQ2
                  + 50 * N_DBL + 70 * N_ADD)
SLOTS_DSM_FINAL = 5 * SLOT_MUL
SLOTS_DSM = SLOTS_DSM_SETUP + SLOTS_DSM_LOOP + SLOTS_DSM_FINAL
# fd_k_decomp, per point (avx/fd_ed25519_ge.c:222-299 + fd_ed25519_ge.c:11-66):
#   264 sq + 3 sq2 (pow22523 251, 4 around it, small-order 3 x 4) and 32 mul,
#   + frombytes 60 + 3 canonical reductions x 40; two points per verify.
SLOTS_DECOMP = 2 * (264 * SLOT_SQ + 3 * SLOT_SQ2 + 32 * SLOT_MUL + 60 + 120)
# fd_k_prep: SHA-512 blocks + S check, sc_reduce (~600) and two wNAF-5
#   recodings (~1,700 each) = 4,000 fixed.
SLOTS_PREP_FIXED = 4000
PEAK_CLOCK_GHZ = 2.4
PEAK_INT32_OPS = 256 * 4 * 32 * PEAK_CLOCK_GHZ * 1e9   # 256 CUs x 4 SIMD x 32 lanes x 2.4 GHz = 78.6 T slots/s


# algorithmic HBM bytes per verify (the txn bytes a signature
# brings, its descriptor and its code)
ALGO_BYTES_PER_SIG = 1260




def load_traffic(path, n_step, kernel, kid):
    """roofline.traffic from a PMC summary (tools/pmc_summary.py), only if it
    was measured on THIS device-code build (fd_ed25519_gpu_kernels_id: the
    kernel sources and flags) and launch size: a summary of another build
    describes kernels that may no longer exist (round-4 verdict)."""
    if not os.path.exists(path):
        return None, "no PMC summary"
    try:
        tr = json.load(open(path))
    except (OSError, ValueError):
        return None, "unreadable PMC summary"
    if tr.get("kernels_id") != kid:
        return None, f"stale: PMC summary of kernels build {tr.get('kernels_id')}, loaded {kid}"
    if tr.get("sigs_per_launch") != n_step:
        return None, f"PMC summary of {tr.get('sigs_per_launch')} signatures per launch, this run {n_step}"
    v = tr.get("kernels", {}).get(kernel, {}).get("hbm_bytes_per_launch")
    return v, ("current" if v is not None else f"no FETCH/WRITE for {kernel}")


def sha_blocks(msg_sz):
    return (64 + msg_sz + 17 + 127) // 128


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--step-batches", type=int, default=STEP_BATCHES)
    ap.add_argument("--unique", type=int, default=0,
                    help="distinct signatures per GPU (0: one per signature of a step, so the timed launches "
                         "never re-read an input that could sit in the 256 MB MALL)")
    ap.add_argument("--no-cpu", action="store_true", help="skip the CPU baseline leg")
    ap.add_argument("--no-latency", action="store_true")
    ap.add_argument("--latency-batches", type=int, default=10000, help="C2 latency: >= 10^4 batches (SURVEY 8d)")
    ap.add_argument("--ring-depth", type=int, default=8, help="ring slots of the C2 streaming leg")
    ap.add_argument("--ring-window", type=int, default=6,
                    help="batches in flight on the C2 streaming leg (below the depth: free slots on the least "
                         "loaded CU group; 6 of 8 keeps p99 under 1 ms, profiles/r02_ring_sweep_contiguous.jsonl)")
    ap.add_argument("--dry-cpu", action="store_true", help="rehearse the multi-rank plumbing on the CPU (tests only)")
    ap.add_argument("--cpu-sample", type=int, default=393216, help="signatures in the CPU baseline sample (~15 thread-s of reference work)")
    ap.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    ap.add_argument("--stream-batches", type=int, default=48,
                    help="batches of the PCIe-inclusive large-batch C2 leg (c2_streamed)")
    return ap.parse_args()


def usable_cores():
    """CPUs this process may actually run on: the affinity mask, capped by
    the cgroup CPU quota (a GPU box grants a job a share of the host: its
    os.cpu_count() is the whole machine)."""
    n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    try:
        q, per = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


def _time_checker(L, fn, sub, threads):
    import ctypes
    sig, pub, data, off, sz = sub.flat()
    out = np.zeros(len(sub), np.int32)
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    t0 = time.perf_counter()
    getattr(L, fn)(ctypes.c_uint64(len(sub)), P(sig), P(pub), P(data), P(off), P(sz), P(out), threads)
    dt = time.perf_counter() - t0
    assert (out == 0).all(), f"CPU baseline ({fn}) rejected valid signatures"
    return dt


def cpu_baseline(batch, nsig, threads):
    """The reference's own fd_ed25519_verify (oracle/_ref/libfdref.so, the
    AVX2 build compiled from /root/reference; 'reference') timed on a
    bounded sample of the same corpus on every core this job may use, plus
    the SURVEY.md 8d calibration ratio: the CPU restatement
    (oracle/liboracle.so) / the reference on the same sample, same box.
    Falls back to the restatement ('port') only if the reference build
    was not shipped, and says so."""
    import ctypes
    ref = os.path.join(ROOT, "oracle", "_ref", "libfdref.so")
    port = os.path.join(ROOT, "oracle", "liboracle.so")
    sub = batch.tile(int(math.ceil(nsig / len(batch))))
    sub.desc = sub.desc[:nsig]
    res = {"unit": "verifies/s", "cores": threads, "cpu": _cpu_model(), "host_cpus_visible": os.cpu_count()}
    if os.path.exists(ref):
        dt = _time_checker(ctypes.CDLL(ref), "ref_verify_batch", sub, threads)
        res.update(value=nsig / dt, kind="reference")
    elif os.path.exists(port):
        dt = _time_checker(ctypes.CDLL(port), "oracle_verify_batch", sub, threads)
        res.update(value=nsig / dt, kind="port", note="reference build not shipped: restatement timed")
    else:
        return None
    res["per_core"] = res["value"] / threads
    # a 4096-signature batch on the CPU = the wall time of 4096 verifies on these cores
    res["batch_4096_ms"] = 4096.0 / res["value"] * 1e3
    res["sample"] = (f"{nsig} signatures of the same C2 corpus (1232-byte txns, msg 1167/1103 B), "
                     f"{threads} host threads (all this job may use), {dt:.2f} s wall ({dt * threads:.1f} thread-s)")
    if res["kind"] == "reference" and os.path.exists(port):
        cal = batch.tile(1)
        cal.desc = cal.desc[:min(len(cal), max(threads * 2048, 16384))]
        t_ref = _time_checker(ctypes.CDLL(ref), "ref_verify_batch", cal, threads)
        t_port = _time_checker(ctypes.CDLL(port), "oracle_verify_batch", cal, threads)
        res["calibration"] = {"restatement_over_reference": t_ref / t_port, "sample_sigs": len(cal),
                              "note": "throughput ratio of the CPU restatement to the reference build, same "
                                      "sample and threads on this box (SURVEY.md 8d)"}
    return res


def step_reference_codes(batch, threads):
    """The reference build's codes for every signature of the step corpus
    (the checker, run after the timed region; None if it was not shipped)."""
    import ctypes
    ref = os.path.join(ROOT, "oracle", "_ref", "libfdref.so")
    if not os.path.exists(ref):
        return None
    sig, pub, data, off, sz = batch.flat()
    exp = np.zeros(len(batch), np.int32)
    P = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    ctypes.CDLL(ref).ref_verify_batch(ctypes.c_uint64(len(batch)), P(sig), P(pub), P(data), P(off), P(sz), P(exp), threads)
    return exp


def reference_check(batch, got, threads, exp=None):
    """The reference's fd_ed25519_verify (oracle/_ref/libfdref.so) over every
    signature of the step corpus, code by code against the engine's codes of
    the first step.  The checker only: nothing timed goes through it."""
    t0 = time.time()
    if exp is None:
        exp = step_reference_codes(batch, threads)
    if exp is None:
        return {"checked": False, "note": "reference build not shipped"}
    mism = int((exp != got[:len(batch)]).sum())
    return {"checked": True, "sigs": len(batch), "mismatches": mism, "reference_codes": codes_hist(exp),
            "seconds": time.time() - t0, "checker": "oracle/_ref/libfdref.so (reference AVX2 build)"}


def _cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def timed_region(step, steps, warmup, dist, red_dev, sync, on_start=None):
    """W untimed warmup steps, then exactly K steps bracketed by a barrier +
    device sync on both sides; returns the MAX over ranks of the wall time."""
    for _ in range(warmup):
        step()
    sync()
    if dist:
        dist.barrier()
    sync()
    if on_start:
        on_start()
    t_start = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    if dist:
        dist.barrier()
    elapsed = time.perf_counter() - t_start
    if dist:
        import torch
        t = torch.tensor([elapsed], dtype=torch.float64, device=red_dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
    return elapsed


def codes_hist(codes):
    u, c = np.unique(np.asarray(codes), return_counts=True)
    return {str(int(k)): int(v) for k, v in zip(u, c)}


def valid_corpus_ok(hist, n):
    """Codes of an all-valid corpus: every signature accepted except the few
    the reference itself rejects through its limb compare (about
    1.4 per million valid signatures, always ERR_MSG)."""
    rej = sum(v for k, v in hist.items() if k != "0")
    return set(hist) <= {"0", "-3"} and rej <= max(4, int(n * 1e-5))


def all_ranks_ok(ok, dist, red_dev):
    if not dist:
        return ok
    import torch
    okt = torch.tensor([1 if ok else 0], device=red_dev)
    dist.all_reduce(okt, op=dist.ReduceOp.MIN)
    return bool(okt.item())


def dry_cpu(a, rank, world):
    """Rehearsal of the N-rank plumbing on the CPU (tests/test_bench_dist.py):
    torch.distributed.run launch, gloo barrier, max-over-ranks timing and
    the whole-job aggregate, with a fixed host step standing in for the
    GPU launch.  Never a measurement: data says so."""
    import torch.distributed as torch_dist
    dist = None
    if world > 1:
        torch_dist.init_process_group("gloo")
        dist = torch_dist
    n_step = a.step_batches * BATCH_SIGS
    x = np.arange(1 << 16, dtype=np.uint64)

    def step():
        np.bitwise_xor.reduce(x * np.uint64(2654435761 + rank))

    elapsed = timed_region(step, a.steps, a.warmup, dist, "cpu", lambda: None)
    ok = all_ranks_ok(True, dist, "cpu")
    res = result_line(a, world, n_step, elapsed, ok, None)
    res["data"] = "dry-cpu rehearsal of the multi-rank plumbing (no GPU, no verification): not a measurement"
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


def result_line(a, world, n_step, elapsed, ok, base, hist=None):
    total = n_step * a.steps * world
    return {
        "metric": "Ed25519 verifies/sec at 1/2/4/8 MI355X; p99 latency per 4096-sig batch",
        "value": total / elapsed,
        "unit": "verifies/s",
        "n_gpus": world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": elapsed / a.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": "synthetic",
        "config": {
            "workload": "C2: 4096-signature batches of 1232-byte Solana legacy txns, 1-2 sigs/txn (p=0.7/0.3), all valid",
            "batch_sigs": BATCH_SIGS,
            "batches_per_step": a.step_batches,
            "sigs_per_step_per_gpu": n_step,
            "unique_sigs_per_gpu": len(base) if base is not None else None,
            "msg_sz": sorted(set(int(x) for x in np.unique(base.desc["msg_sz"]))) if base is not None else None,
            "parallelism": f"replicas x{world} (independent per-GPU shards, no collective)",
        },
        "codes_ok": ok,
        "codes": hist,
    }


def main():
    a = parse()
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if a.dry_cpu:
        return dry_cpu(a, rank, world)
    import torch
    dist = None
    # rehearsal only (FD_BENCH_SHARE_GPU=1): more ranks than GPUs share them,
    # with gloo carrying the barrier and the max-over-ranks
    share = os.environ.get("FD_BENCH_SHARE_GPU") == "1"
    if share:
        local = local % max(1, torch.cuda.device_count())
    red_dev = "cpu" if share else torch.device("cuda", local)
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        if share:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(local)

    import firedancer_amd as fa
    from firedancer_amd import corpus

    n_step = a.step_batches * BATCH_SIGS
    t0 = time.time()
    base = corpus.solana_txns(a.unique or n_step, seed=1000 + rank, nthreads=min(16, os.cpu_count() or 8))
    batch = base.tile(int(math.ceil(n_step / len(base))))
    batch.desc = batch.desc[:n_step]
    gen_s = time.time() - t0

    eng = fa.Engine(local, max_sigs=max(n_step, 1 << 16), max_blob=max(len(batch.blob), 1 << 24))
    dev = torch.device("cuda", local)
    blob_sz = len(batch.blob)
    d_blob = torch.from_numpy(np.concatenate([batch.blob, np.zeros(64, np.uint8)])).to(dev)
    d_desc = torch.from_numpy(batch.desc.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n_step, dtype=torch.int32, device=dev)
    stream = torch.cuda.current_stream(dev).cuda_stream

    torch.cuda.synchronize()     # the inputs are resident and complete before the timed region
    overlap = os.environ.get("FD_BENCH_SERIAL") != "1"     # A/B: serial launches

    def step():
        eng.verify_dev(n_step, d_blob.data_ptr(), blob_sz, d_desc.data_ptr(), d_out.data_ptr(), stream, inputs_ready=overlap)

    # the first warmup step's codes are checked (all valid: all accepted)
    step()
    torch.cuda.synchronize()
    hist = codes_hist(d_out.cpu().numpy())
    ok = valid_corpus_ok(hist, n_step)
    solo = rank == 0 and world == 1
    def on_start():
        eng.dev_stats_begin()
        eng.dsm_clock(clear=True)
    elapsed = timed_region(step, a.steps, max(a.warmup - 1, 0), dist, red_dev, torch.cuda.synchronize,
                           on_start=on_start if solo else None)
    live = eng.dev_stats_end() if solo else None
    clock = eng.dsm_clock() if solo else None
    ok = all_ranks_ok(ok, dist, red_dev)
    res = result_line(a, world, n_step, elapsed, ok, base, hist)
    value = res["value"]

    if solo:
        # per-kernel durations LIVE over the timed launches: HIP events around
        # each kernel on the stream it runs on (the device-resident pipeline
        # overlaps launch k's front end with launch k-1's DSM)
        ks, timed_launches = live
        # and each kernel alone (serial launches), for the breakdown
        reps = max(3, min(a.steps, 10))
        ks_serial = np.zeros(len(fa.Engine.KERNELS))
        for _ in range(reps):
            ks_serial += eng.verify_dev_timed(n_step, d_blob.data_ptr(), blob_sz, d_desc.data_ptr(), d_out.data_ptr(), stream)
        ks_serial /= reps
        msz = base.desc["msg_sz"].astype(np.int64)
        blocks = float(np.mean([sha_blocks(int(m)) for m in msz]))
        ops = {"fd_k_prep": (SLOT_SHA_BLOCK * blocks + SLOTS_PREP_FIXED) * n_step,
               "fd_k_decomp": SLOTS_DECOMP * n_step,
               "fd_k_dsm_setup": SLOTS_DSM_SETUP * n_step,
               "fd_k_dsm_pool": SLOTS_DSM_LOOP * n_step,
               "fd_k_dsm_final": SLOTS_DSM_FINAL * n_step}
        kern = {}
        for name, ms, ms1 in zip(fa.Engine.KERNELS, ks, ks_serial):
            ach = ops[name] / (ms * 1e-3) / 1e12 if ms > 0 else 0.0
            ach1 = ops[name] / (ms1 * 1e-3) / 1e12 if ms1 > 0 else 0.0
            # live ms of the front-end kernels include time they wait on the SIMDs of the
            # previous launch's DSM (which runs at a higher stream priority); frac_serial
            # is each kernel alone
            kern[name] = {"ms": float(ms), "achieved_Tops": ach, "frac": ach * 1e12 / PEAK_INT32_OPS,
                          "ms_serial": float(ms1), "frac_serial": ach1 * 1e12 / PEAK_INT32_OPS}
        dom = max(kern, key=lambda k: kern[k]["ms_serial"])     # the kernel with the most work
        traffic, traffic_status = load_traffic(a.traffic, n_step, dom, fa.kernels_id())
        w_total = SLOTS_DSM + SLOTS_DECOMP + SLOT_SHA_BLOCK * blocks + SLOTS_PREP_FIXED
        res["roofline"] = {
            "bound": "valu-int32",
            "kernel": dom,
            "achieved": kern[dom]["achieved_Tops"],
            "peak": PEAK_INT32_OPS / 1e12,
            "unit": "Tint32op/s",
            "frac": kern[dom]["frac"],
            "traffic": traffic,
            # HBM bytes the kernel moved / the path's algorithmic bytes for the
            # signatures of one launch (1.26 KB per verify -- the
            # txn bytes, descriptors and codes; every intermediate stays on chip
            # in the model)
            "traffic_ratio": None if traffic is None else traffic / (ALGO_BYTES_PER_SIG * n_step),
            "traffic_status": traffic_status,
            "per_kernel": kern,
            "pipeline_frac": value * w_total / PEAK_INT32_OPS,
            # the shader clock the pool ran at over the timed launches (s_memtime vs
            # the 100 MHz s_memrealtime, summed over its waves): the peak assumes
            # 2.4 GHz, so boxes whose DVFS holds a lower clock under this load
            # read a lower frac for the same code
            "effective_clock_ghz": clock["pool"]["ghz"],
            "frac_at_effective_clock": (kern[dom]["frac"] * PEAK_CLOCK_GHZ / clock["pool"]["ghz"]
                                        if clock["pool"]["ghz"] else None),
            "clock_source": "fd_ed25519_gpu_dsm_clock: fd_k_dsm_pool waves' s_memtime / s_memrealtime "
                            f"over the timed launches ({clock['pool']['waves']} waves)",
            "ops_per_verify": w_total,
            "kernel_ms_source": f"HIP events around each kernel on its stream over {timed_launches} timed launches "
                                "(pipelined: launch k's front end overlaps launch k-1's DSM); ms_serial: each "
                                "kernel alone (fd_ed25519_gpu_verify_dev_timed)",
            "work_model": "reference field-op / SHA-block counts x minimal gfx950 issue slots "
                          "(MAC and 64-bit ops 2, int32 op 1); peak = 78.6 T full-rate int32 lane-op "
                          "slots/s (DESIGN.md section 4)",
            "traffic_note": "HBM bytes per launch of the dominant kernel from rocprofv3 PMC "
                            "(2*FETCH_SIZE + WRITE_SIZE, profiles/pmc_traffic.json, used only when "
                            "its recorded library hash equals the loaded library's); the path is "
                            "VALU-bound, traffic is a secondary check",
        }
        if not a.no_latency:
            eng.dsm_clock(clear=True)
            res["latency"] = latency_legs(fa, corpus, a, local)
            lat = res["latency"]
            torch.cuda.synchronize()
            qc = eng.dsm_clock()["quad"]
            lat["dsm_quad_effective_clock_ghz"] = qc["ghz"]
            lat["dsm_quad_clock_waves"] = qc["waves"]
            res["ring_4096_verifies_per_s"] = lat["pcie_inclusive_verifies_per_s"]
            res["ring_4096_best_verifies_per_s_at_p99_le_1ms"] = (lat["best_under_p99_1ms"] or {}).get("verifies_per_s")
            res["ring_4096_max_offered_at_sched_p99_le_1ms"] = lat["max_offered_at_sched_p99_le_1ms"]
        step_codes = d_out.cpu().numpy()
        exp_step = step_reference_codes(batch, usable_cores())
        if not a.no_latency:
            # the deployable C2 number: the same step corpus streamed from host
            # memory through the feeder and the registered ring at pool
            # granularity, PCIe both ways included (the `value` is HBM-resident)
            big = ring_stream(fa, batch, local, a.stream_batches, 3, window=3, expected=exp_step,
                              batch_sigs=STREAM_BATCH_SIGS, q2_at=())
            big["content"] = ("the step corpus (C2: 1232-byte txns, 1-2 sigs/txn), batches of "
                              f"{STREAM_BATCH_SIGS} signatures DMA'd from a registered host region, codes to the host")
            res["c2_streamed"] = big
            res["c2_streamed_large_batch_verifies_per_s"] = big["pcie_inclusive_verifies_per_s"] if big["codes_ok"] else None
        if not a.no_cpu:
            res["cpu_baseline"] = cpu_baseline(base, a.cpu_sample, usable_cores())
            # the checker: the reference build's codes for the whole step corpus
            # vs the engine's (the rejects above are the reference's own)
            res["reference_check"] = reference_check(batch, step_codes, usable_cores(), exp_step)
        res["corpus_gen_s"] = gen_s

    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist:
        dist.destroy_process_group()


# the C2 ring's corpus: RING_WINDOWS windows of one batch each, the C3 mix
# (10 % invalid over every case of corpus.CASES) plus the three SURVEY Q2
# vectors at fixed offsets of every window (only a limb-exact engine rejects
# them), so every timed ring batch carries reference evidence
RING_WINDOWS = 64
RING_Q2_AT = (1024, 2048, 4095)
# the PCIe-inclusive C2 leg at pool granularity (c2_streamed)
STREAM_BATCH_SIGS = 262144
# offered loads of the open-loop sweep, M verifies/s
PACED_MPS = (25, 30, 32, 34, 36, 38, 40)


def ring_reference_codes(ring, threads):
    """The reference build's codes for the ring corpus (the checker; computed
    before the ring legs, compared with each leg's codes after it is timed)."""
    import ctypes
    ref = os.path.join(ROOT, "oracle", "_ref", "libfdref.so")
    if not os.path.exists(ref):
        return None
    sig, pub, data, off, sz = ring.flat()
    exp = np.zeros(len(ring), np.int32)
    P = lambda x: x.ctypes.data_as(ctypes.c_void_p)  # noqa: E731
    ctypes.CDLL(ref).ref_verify_batch(ctypes.c_uint64(len(ring)), P(sig), P(pub), P(data), P(off), P(sz), P(exp), threads)
    return exp


def latency_legs(fa, corpus, a, device):
    """C2 at its own granularity, PCIe both ways: closed-loop points (batches
    outstanding 5-8 on a depth-8 ring, depth 4, depth 1) and an open-loop
    sweep of offered loads (PACED_MPS) whose latency is scheduled arrival ->
    codes on the host.  Every code of every leg is compared with the
    reference build's after the leg."""
    t0 = time.time()
    ring = corpus.c3_windows(RING_WINDOWS, BATCH_SIGS, seed=4242, extra=[
        (bytes.fromhex(m), bytes.fromhex(s), bytes.fromhex(p)) for m, s, p in corpus.Q2_VECTORS],
        extra_at=RING_Q2_AT, nthreads=min(16, os.cpu_count() or 8))
    gen_s = time.time() - t0
    t0 = time.time()
    exp = ring_reference_codes(ring, usable_cores())
    ref_s = time.time() - t0
    global RING_CORES
    RING_CORES = tuple(fa.quiet_cpus(2, device)) or None
    nb, nb2 = a.latency_batches, max(a.latency_batches // 2, 20)
    lat = ring_stream(fa, ring, device, nb, a.ring_depth, window=a.ring_window, expected=exp)
    lat["corpus"] = {"windows": RING_WINDOWS, "sigs": len(ring), "q2_at": list(RING_Q2_AT), "gen_s": gen_s,
                     "reference_codes": None if exp is None else codes_hist(exp), "reference_s": ref_s,
                     "content": "C3 mix at C2 shape: 1232-byte txns, 10 % of the signatures corrupted over all 18 "
                                "invalid cases, the 3 SURVEY Q2 vectors at fixed offsets of every 4096-signature window"}
    # closed loop: more / fewer batches outstanding, a shallower ring, one at a time
    lat["throughput_point"] = ring_stream(fa, ring, device, nb2, a.ring_depth, window=min(a.ring_window + 1, a.ring_depth),
                                          expected=exp)
    lat["window5_point"] = ring_stream(fa, ring, device, nb2, a.ring_depth, window=max(a.ring_window - 1, 1), expected=exp)
    lat["window8_point"] = ring_stream(fa, ring, device, nb2, a.ring_depth, window=a.ring_depth, expected=exp)
    lat["lower_latency_point"] = ring_stream(fa, ring, device, nb2, 4, expected=exp)
    lat["depth1"] = ring_stream(fa, ring, device, max(nb // 5, 20), 1, expected=exp)
    pts = [lat] + [lat[k] for k in ("throughput_point", "window5_point", "window8_point", "lower_latency_point", "depth1")]
    ok = [p for p in pts if p["p99_ms"] <= 1.0 and p["codes_ok"]]
    best = max(ok, key=lambda p: p["pcie_inclusive_verifies_per_s"]) if ok else None
    lat["best_under_p99_1ms"] = None if best is None else {
        "verifies_per_s": best["pcie_inclusive_verifies_per_s"], "p99_ms": best["p99_ms"], "p50_ms": best["p50_ms"],
        "window": best["window"], "ring_depth": best["ring_depth"], "latency": "push -> codes on the host (closed loop)"}
    # open loop: one batch every period_ns, latency from its scheduled arrival
    # (a batch the full ring holds back waits, and that wait is counted)
    paced = []
    for mps in PACED_MPS:
        # up to 2 x depth outstanding: the feeder always holds the next batch
        # when a slot frees; what the ring cannot take waits in its queue
        # and that wait is part of sched -> done
        # each offered load over the full >= 10^4 batches (C2's
        # p50 / p99 over at least 10^4 batches; round 4 ran half of that)
        r = ring_stream(fa, ring, device, nb, a.ring_depth, window=2 * a.ring_depth,
                        period_ns=int(round(BATCH_SIGS / (mps * 1e6) * 1e9)), expected=exp)
        paced.append(r)
    lat["paced"] = paced
    held = [r for r in paced if r["sustained"] and r["sched_to_done_p99_ms"] <= 1.0 and r["codes_ok"]]
    top = max(held, key=lambda r: r["offered_verifies_per_s"]) if held else None
    lat["max_offered_at_sched_p99_le_1ms"] = None if top is None else top["offered_verifies_per_s"]
    lat["max_offered_point"] = None if top is None else {
        k: top[k] for k in ("offered_verifies_per_s", "pcie_inclusive_verifies_per_s", "sched_to_done_p50_ms",
                            "sched_to_done_p99_ms", "p99_ms", "mismatches")}
    return lat


# the ring legs' two spinning host threads (the synthetic producer, the
# per-GPU feeder) each on a quiet core of the GPU's NUMA node, as a
# validator pins its tiles (fa.quiet_cpus); chosen once per run
RING_CORES = None


def ring_stream(fa, base, device, nb, depth, groups=None, window=None, register=True, seed=7, period_ns=0,
                expected=None, batch_sigs=BATCH_SIGS, q2_at=RING_Q2_AT):
    """C2 at its own granularity: nb 4096-signature batches streamed through
    one engine's pinned ring by its per-GPU feeder thread
    (fd_ed25519_gpu_feeder: NUMA-pinned, whole ring in flight), PCIe both
    ways included.  The corpus blob is registered with the engine (as a
    tile registers its input dcache), so a batch is DMA'd from where it
    lies with no staging memcpy.  The producer is the library's native
    synthetic-load loop (fd_ed25519_gpu_feeder_synth, the counterpart of
    the reference's synth-load verify tile): `window` batches outstanding
    (closed loop; latency = push -> codes on the host), or one batch pushed
    every period_ns (paced, at most `window` outstanding; latency =
    scheduled arrival -> codes on the host).  Batch i is window
    starts[i % 64] of `base` (one batch per BATCH_SIGS-signature window);
    every code is returned and, with `expected` (the reference build's codes
    for `base`), compared code by code after the timed run."""
    BS = batch_sigs
    nwin = len(base) // BS
    # the largest blob span of a window (a batch moves one span)
    span = 8 << 20
    for w in range(nwin):
        d = base.desc[w * BS:(w + 1) * BS]
        lo = int(min(d["sig_off"].min(), d["pub_off"].min(), d["msg_off"].min()))
        hi = int(max((d["sig_off"].astype(np.int64) + 64).max(), (d["pub_off"].astype(np.int64) + 32).max(),
                     (d["msg_off"].astype(np.int64) + d["msg_sz"]).max()))
        span = max(span, hi - lo + 64)
    eng = fa.Engine(device, max_sigs=BS, max_blob=span, depth=depth)
    prev_aff = os.sched_getaffinity(0)
    cores = RING_CORES
    try:
        if groups:
            eng.cu_groups = groups
        if register:
            eng.register(base.blob)
        # the feeder thread takes the creating thread's CPUs (within the
        # GPU's NUMA node); then this thread, the producer, moves to its own
        if cores:
            os.sched_setaffinity(0, {cores[1]})
        feeder = fa.Feeder(eng)
        if cores:
            os.sched_setaffinity(0, {cores[0]})
        starts = np.random.default_rng(seed).permutation(nwin).astype(np.uint64) * BS
        W = window or depth
        # untimed warm-up: two closed-loop passes over every window, so the
        # engine's first launches on each slot's CU-group stream and the
        # first DMA of each page of the freshly registered corpus are not
        # inside the measured stream (tools/ring_paced_tail.py saw a
        # ~20 ms stall in a fresh engine's first 60 ms)
        feeder.synth(base.blob, base.desc, BS, starts, 2 * nwin, depth, 0)
        t0 = time.perf_counter()
        st, codes = feeder.synth(base.blob, base.desc, BS, starts, nb, W, period_ns, codes=True)
        wall = time.perf_counter() - t0
        numa = feeder.numa_node
        feeder.close()
        # the codes of EVERY batch (fill included) against the reference
        c = st["codes"].sum(axis=0)
        hist = {k: int(v) for k, v in zip(("0", "-1", "-2", "-3", "other"), c) if v or k == "0"}
        complete = bool((st["state"] == 1).all()) and int(c.sum()) == nb * BS and int(c[4]) == 0
        mism = None
        label_mism = None
        if expected is not None:
            mism = 0
            for s in range(min(len(starts), nb)):
                rows = codes[s::len(starts)]
                o = int(starts[s])
                mism += int((rows != expected[o:o + BS][None, :]).sum())
        elif base.label is not None:
            # no reference build on this box: the corpus's own labels, which
            # decide only the untouched signatures (valid, label 0, off the
            # Q2 offsets) -- a partial check, so codes_ok stays None
            label_mism = 0
            keep = np.ones(BS, bool)
            keep[list(q2_at)] = False
            for s in range(min(len(starts), nb)):
                rows = codes[s::len(starts)]
                o = int(starts[s])
                v = (base.label[o:o + BS] == 0) & keep
                label_mism += int((rows[:, v] != 0).sum())
        skip = W if nb > 2 * W else 0          # the ring's fill
        st = st[skip:]
        lat = (st["t_done_ns"] - st["t_push_ns"]) * 1e-6
        qlat = (st["t_done_ns"] - st["t_submit_ns"]) * 1e-6
        hop = (st["t_submit_ns"] - st["t_push_ns"]) * 1e-6
        pick = (st["t_pick_ns"] - st["t_push_ns"]) * 1e-6      # the feeder's pickup
        enq = (st["t_submit_ns"] - st["t_pick_ns"]) * 1e-6     # staging + HIP enqueue of the batch
        res = {"batch_sigs": BS, "batches": nb, "ring_depth": depth, "window": W,
               "cu_groups": eng.cu_groups, "registered_source": bool(register),
               "feeder_numa_node": numa, "producer": "native (fd_ed25519_gpu_feeder_synth)",
               "pcie_inclusive_verifies_per_s": nb * BS / wall,
               "p50_ms": float(np.percentile(lat, 50)), "p99_ms": float(np.percentile(lat, 99)),
               "p999_ms": float(np.percentile(lat, 99.9)), "max_ms": float(lat.max()),
               "submit_to_done_p50_ms": float(np.percentile(qlat, 50)),
               "submit_to_done_p99_ms": float(np.percentile(qlat, 99)),
               "push_to_submit_p50_ms": float(np.percentile(hop, 50)),
               "push_to_submit_p99_ms": float(np.percentile(hop, 99)),
               "push_to_pick_p50_ms": float(np.percentile(pick, 50)), "push_to_pick_p99_ms": float(np.percentile(pick, 99)),
               "pick_to_submit_p50_ms": float(np.percentile(enq, 50)), "pick_to_submit_p99_ms": float(np.percentile(enq, 99)),
               "codes": hist, "reference_checked": expected is not None, "mismatches": mism,
               "label_check_mismatches": label_mism,
               # True only when every code was compared with the reference build's
               "codes_ok": (complete and mism == 0) if expected is not None else (False if not complete else None),
               "host_cores": None if not cores else {"producer": cores[0], "feeder": cores[1]}}
        if period_ns:
            sl = (st["t_done_ns"] - st["t_sched_ns"]) * 1e-6
            offered = BS / (period_ns * 1e-9)
            res.update(offered_verifies_per_s=offered,
                       sustained=res["pcie_inclusive_verifies_per_s"] >= 0.98 * offered,
                       sched_to_done_p50_ms=float(np.percentile(sl, 50)),
                       sched_to_done_p99_ms=float(np.percentile(sl, 99)),
                       sched_to_done_max_ms=float(sl.max()),
                       latency="scheduled arrival -> codes on the host (p50_ms/p99_ms: push -> codes)")
        return res
    finally:
        os.sched_setaffinity(0, prev_aff)
        eng.close()


if __name__ == "__main__":
    main()
