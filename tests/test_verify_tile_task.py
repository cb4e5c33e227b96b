"""The verify tile as a task (fd_verify_tile_task, include/fd_verify_tile.h)
with the reference tile's shape and run loop (src/app/frank/fd_frank.h:29-45,
src/app/frank/fd_frank_verify.c:7-205): init creates all device state and
reports the seccomp allowlist; run handles the cnc (RUN, HALT -> drain ->
BOOT), heartbeat, flow-control backpressure (IN_BACKP / BACKP_CNT) and the
frag path; publish decisions and counters equal the reference's per-frag
semantics (fd_frank_verify_synth_load.c:360-410) with every signature
checked by the reference's own fd_ed25519_verify."""
import json
import os
import struct
import subprocess
import threading
import time

import pytest

import firedancer_amd as fa
from conftest import ROOT
from firedancer_amd import tile as T

from test_verify_tile import expected_for, make_stream

REFERENCE_ALLOW = {1, 202, 74, 35}   # __NR_write, futex, fsync, nanosleep (fd_frank_verify.c:7-12, x86-64)


def test_task_shape_and_allowlist_without_gpu():
    """init reports the reference's four syscalls plus what HIP needs; with
    no gfx950 device it fails loudly (cnc FAIL), never falls back"""
    if fa.device_count() > 0:
        pytest.skip("a gfx950 device is present")
    t = T.Task([], device=0)
    assert t.name == "verify"
    err = t.init()
    assert err == fa.ERR_GPU
    assert t.cnc.signal == T.SIGNAL_FAIL
    allow = set(t.allow_syscalls())
    assert REFERENCE_ALLOW <= allow
    assert {16, 9, 11, 10, 24} <= allow          # ioctl, mmap, munmap, mprotect, sched_yield
    assert t.args.close_fd_start == 4


def _run_task(task, halt_when_drained=True, timeout=60.0):
    """run on a thread; HALT once every frag was taken (as a cnc thread would)"""
    res = {}
    th = threading.Thread(target=lambda: res.setdefault("err", task.run()))
    th.start()
    t0 = time.time()
    while halt_when_drained and task.next < len(task.frags) and time.time() - t0 < timeout:
        time.sleep(0.005)
    time.sleep(0.01)
    task.halt()
    th.join(timeout)
    assert not th.is_alive(), "run loop did not stop on HALT"
    return res["err"]


@pytest.mark.gpu
def test_task_stream_vs_reference(ref):
    frags = make_stream(4000, 77, ref)
    exp_pub, exp, nsig = expected_for(frags, ref)
    task = T.Task(frags, batch_sigs=1024)
    assert task.init() == 0
    assert task.cnc.signal == T.SIGNAL_BOOT
    try:
        assert _run_task(task) == 0
        assert task.cnc.signal == T.SIGNAL_BOOT            # HALT acknowledged (fd_cnc.h:40-43)
        assert task.cnc.heartbeat > 0
        assert [(s, f) for s, f, _, _ in task.published] == exp_pub
        d = task.diag()
        for k, v in exp.items():
            assert d[k] == v, k
        assert d["PUB_CNT"] == len(exp_pub) and d["SIG_CNT"] == nsig
        assert d["IN_BACKP"] == 0 and d["BACKP_CNT"] == 0
    finally:
        task.fini()


@pytest.mark.gpu
def test_task_multi_engine_vs_reference(ref):
    """device_cnt = 2: the task makes one engine per device (both on this
    box's one GPU) and runs the tile in feeder mode; same publishes and
    counters as the reference's per-frag semantics"""
    frags = make_stream(3000, 79, ref)
    exp_pub, exp, nsig = expected_for(frags, ref)
    task = T.Task(frags, batch_sigs=512, max_sigs=1024, max_blob=4 << 20, depth=2, device_cnt=2)
    assert task.init() == 0
    try:
        assert task.args.gpus[0] and task.args.gpus[1] and task.args.gpu == task.args.gpus[0]
        assert _run_task(task) == 0
        assert task.cnc.signal == T.SIGNAL_BOOT
        assert [(s, f) for s, f, _, _ in task.published] == exp_pub
        d = task.diag()
        for k, v in exp.items():
            assert d[k] == v, k
        assert d["PUB_CNT"] == len(exp_pub) and d["SIG_CNT"] == nsig
    finally:
        task.fini()
    assert not task.args.gpu and not task.args.gpus[1]


@pytest.mark.gpu
def test_task_backpressure_diag(ref):
    """no downstream credits for the first housekeeping rounds: IN_BACKP set
    and BACKP_CNT counted (fd_frank_verify.c:185-194), then the stream
    completes once credits return"""
    frags = make_stream(600, 78, ref)
    exp_pub, _, _ = expected_for(frags, ref)
    calls = {"n": 0}

    def credits(task):
        calls["n"] += 1
        return 0 if 3 <= calls["n"] < 12 else 1 << 40

    task = T.Task(frags, credits=credits, lazy_ns=200_000)
    assert task.init() == 0
    try:
        assert _run_task(task) == 0
        d = task.diag()
        assert d["BACKP_CNT"] >= 1 and d["IN_BACKP"] == 0
        assert [(s, f) for s, f, _, _ in task.published] == exp_pub
    finally:
        task.fini()


@pytest.mark.gpu
def test_task_bad_signal_fails():
    """any cnc signal other than RUN / HALT while running -> FAIL (the
    reference logs an error and exits, fd_frank_verify.c:170-173)"""
    task = T.Task([])
    assert task.init() == 0
    try:
        th = threading.Thread(target=task.run)
        th.start()
        time.sleep(0.05)
        task.cnc.signal = 7
        th.join(30)
        assert not th.is_alive()
        assert task.cnc.signal == T.SIGNAL_FAIL and task.args.err != 0
    finally:
        task.fini()


@pytest.mark.gpu
def test_task_under_seccomp(ref, tmp_path):
    """the whole run loop under a seccomp filter allowing exactly the
    task's reported list on every thread (tests/task_seccomp.c): no
    syscall outside it, and the publish stream equals the reference's"""
    exe = os.path.join(ROOT, "firedancer_amd", "test_task_seccomp")
    assert os.path.exists(exe), "build with make -C firedancer_amd"
    frags = make_stream(3000, 79, ref)
    exp_pub, exp, _ = expected_for(frags, ref)
    p = tmp_path / "frags.bin"
    with open(p, "wb") as f:
        f.write(struct.pack("<I", len(frags)))
        for fr in frags:
            f.write(struct.pack("<I", len(fr)) + fr)
    h = 1469598103934665603
    for tag, fr in exp_pub:
        for byte in struct.pack("<QQ", tag, len(fr)):
            h = ((h ^ byte) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    r = subprocess.run([exe, str(p)], capture_output=True, text=True, timeout=120)
    line = r.stdout.strip().splitlines()[-1] if r.stdout.strip() else ""
    assert line, (r.returncode, r.stderr[-2000:])
    out = json.loads(line)
    assert "sigsys" not in out, f"syscall {out.get('sigsys')} outside the tile's allowlist"
    assert r.returncode == 0 and out["err"] == 0, (out, r.stderr[-2000:])
    assert out["signal"] == T.SIGNAL_BOOT
    assert out["pub_cnt"] == len(exp_pub) and int(out["pub_hash"], 16) == h
    d = dict(zip(T.DIAG, out["diag"]))
    for k, v in exp.items():
        assert d[k] == v, k
