#!/usr/bin/env python3
"""Where the paced C2 ring's sched -> done tail comes from: one offered load
(bench.ring_stream's open loop: a 4,096-signature batch every period on the
depth-8 ring, C3-mix corpus), every job's stamps split into
  sched -> push    the producer's own lateness
  push -> pick     the feeder thread taking the job
  pick -> submit   a free ring slot (full ring: waiting for a completion)
                   + staging and enqueue
  submit -> done   H2D, front end, DSM, codes on the host, the feeder
                   noticing
with p50 / p99 of each and the mean of each over the slowest 1 % of jobs.
usage: ring_paced_tail.py [M verifies/s (36)] [batches (4000)] [depth (8)]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def host_stats():
    """CPU-quota throttling and preemption counters of this process's box
    (cgroup v2 or v1 cpu.stat, /proc/pressure/cpu, involuntary context
    switches): a host that stops the feeder thread shows here"""
    import resource
    out = {}
    for f in ("/sys/fs/cgroup/cpu.stat", "/sys/fs/cgroup/cpu/cpu.stat", "/sys/fs/cgroup/cpu,cpuacct/cpu.stat"):
        try:
            for line in open(f):
                k, v = line.split()
                out["cg_" + k] = int(v)
            out["cg_file"] = f
            break
        except (OSError, ValueError):
            pass
    try:
        for line in open("/proc/pressure/cpu"):
            parts = line.split()
            out["psi_" + parts[0] + "_total_us"] = int(parts[-1].split("=")[1])
    except (OSError, ValueError, IndexError):
        pass
    ru = resource.getrusage(resource.RUSAGE_SELF)
    out["nivcsw"] = ru.ru_nivcsw
    out["nvcsw"] = ru.ru_nvcsw
    return out


def main():
    mps = float(sys.argv[1]) if len(sys.argv) > 1 else 36.0
    nb = int(sys.argv[2]) if len(sys.argv) > 2 else 4000
    depth = int(sys.argv[3]) if len(sys.argv) > 3 else 8
    import torch  # noqa: F401  (one HIP runtime)
    import bench
    import firedancer_amd as fa
    from firedancer_amd import corpus
    ring = corpus.c3_windows(bench.RING_WINDOWS, bench.BATCH_SIGS, seed=4242, nthreads=min(16, os.cpu_count() or 8))
    eng = fa.Engine(0, max_sigs=bench.BATCH_SIGS, max_blob=8 << 20, depth=depth)
    eng.register(ring.blob)
    feeder = fa.Feeder(eng)
    B = bench.BATCH_SIGS
    starts = np.random.default_rng(7).permutation(len(ring) // B).astype(np.uint64) * B
    period = int(round(B / (mps * 1e6) * 1e9))
    feeder.synth(ring.blob, ring.desc, B, starts, 400, 2 * depth, period)     # warm-up (first use of every slot and group)
    h0 = host_stats()
    st = feeder.synth(ring.blob, ring.desc, B, starts, nb, 2 * depth, period)
    h1 = host_stats()
    feeder.close()
    eng.close()
    st = st[2 * depth:]
    comp = {
        "sched_to_push": (st["t_push_ns"].astype(np.int64) - st["t_sched_ns"].astype(np.int64)) * 1e-6,
        "push_to_pick": (st["t_pick_ns"].astype(np.int64) - st["t_push_ns"].astype(np.int64)) * 1e-6,
        "pick_to_submit": (st["t_submit_ns"].astype(np.int64) - st["t_pick_ns"].astype(np.int64)) * 1e-6,
        "submit_to_done": (st["t_done_ns"].astype(np.int64) - st["t_submit_ns"].astype(np.int64)) * 1e-6,
    }
    tot = (st["t_done_ns"].astype(np.int64) - st["t_sched_ns"].astype(np.int64)) * 1e-6
    slow = tot >= np.percentile(tot, 99)
    out = {"offered_mps": mps, "batches": int(len(st)), "depth": depth,
           "sched_to_done": {"p50": float(np.percentile(tot, 50)), "p99": float(np.percentile(tot, 99)), "max": float(tot.max())}}
    for k, v in comp.items():
        out[k] = {"p50": float(np.percentile(v, 50)), "p99": float(np.percentile(v, 99)), "slow1pct_mean": float(v[slow].mean())}
    # completions per 1 ms bin: a host stall shows as an empty bin while jobs are outstanding
    done = np.sort(st["t_done_ns"].astype(np.int64))
    gaps = np.diff(done) * 1e-6
    out["completion_gap_ms"] = {"p50": float(np.percentile(gaps, 50)), "p99": float(np.percentile(gaps, 99)), "max": float(gaps.max())}
    # around the worst job: per 5 ms of its scheduled time, jobs completed,
    # the ring's carried rate and the mean submit -> done (a slower ring or
    # a host stall shows here)
    t0 = int(st["t_sched_ns"][0])
    ts = (st["t_sched_ns"].astype(np.int64) - t0) * 1e-6
    td = (st["t_done_ns"].astype(np.int64) - t0) * 1e-6
    w = int(np.argmax(tot))
    lo = max(0.0, ts[w] - 60.0)
    rows = []
    for b0 in np.arange(lo, ts[w] + 20.0, 5.0):
        m = (td >= b0) & (td < b0 + 5.0)
        rows.append([round(float(b0 - ts[w]), 1), int(m.sum()), round(float(m.sum()) * B / 5e-3 / 1e6, 2),
                     round(float(comp["submit_to_done"][m].mean()), 3) if m.any() else None])
    out["around_worst"] = {"cols": ["t_rel_ms", "done", "carried_Mps", "submit_to_done_ms"], "rows": rows}
    out["host_delta"] = {k: h1[k] - h0[k] for k in h1 if isinstance(h1[k], int) and k in h0}
    out["host_cg_file"] = h1.get("cg_file")
    # 2 ms windows of the run that completed less than half the offered rate
    # while jobs were outstanding (a stall of the ring or of the host)
    sched = np.sort(ts)
    stalls = []
    for b0 in np.arange(0.0, float(td.max()), 2.0):
        done_b = int(((td >= b0) & (td < b0 + 2.0)).sum())
        outstanding = int((ts < b0).sum()) - int((td < b0).sum())
        if outstanding > 0 and done_b * B / 2e-3 < 0.5 * mps * 1e6:
            stalls.append([round(float(b0), 1), done_b, outstanding])
    out["slow_2ms_windows"] = stalls[:40]
    out["slow_2ms_window_count"] = len(stalls)
    del sched
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
