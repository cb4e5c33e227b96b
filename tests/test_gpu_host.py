"""Host-runtime behaviour on the GPU (round 3):

  - the engine's two locks are never taken in opposite orders: the
    diagnostic k path (debug_k) and device-resident launches (verify_dev)
    from two threads at once finish (debug_k took g->lock then
    dev_lock while verify_dev held dev_lock and read the knobs under
    g->lock);
  - the live per-kernel timing of pipelined launches attributes the DSM
    setup and the pool to their own streams' events (the back
    part re-recorded the front's ev[3]);
  - the native synthetic-load producer (fd_ed25519_gpu_feeder_synth, the
    bench's C2 ring driver) returns every batch's codes, closed loop and
    paced, equal to the reference's."""
import threading
import time

import numpy as np
import pytest
import torch

import firedancer_amd as fa
from conftest import oracle_batch
from firedancer_amd import corpus

pytestmark = pytest.mark.gpu


def test_debug_k_and_verify_dev_concurrently(ref):
    b = corpus.solana_txns(8192, seed=31)
    exp = oracle_batch(ref, b)
    e = fa.Engine(0, 1 << 14, 1 << 24)
    dev = torch.device("cuda", 0)
    d_blob = torch.from_numpy(np.concatenate([b.blob, np.zeros(64, np.uint8)])).to(dev)
    d_desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(len(b), dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    errs, done = [], [0, 0]
    stop = time.time() + 8.0

    def launches():
        try:
            st = torch.cuda.Stream(dev)
            while time.time() < stop:
                e.verify_dev(len(b), d_blob.data_ptr(), len(b.blob), d_desc.data_ptr(), d_out.data_ptr(), st.cuda_stream)
                st.synchronize()
                assert (d_out.cpu().numpy() == exp).all()
                done[0] += 1
        except Exception as x:     # noqa: BLE001
            errs.append(x)

    def ks():
        try:
            while time.time() < stop:
                k, st = e.debug_k(b.blob[:1 << 20], b.desc[:256])
                assert (st != 0).any()
                done[1] += 1
        except Exception as x:     # noqa: BLE001
            errs.append(x)

    th = [threading.Thread(target=launches, daemon=True), threading.Thread(target=ks, daemon=True)]
    for t in th:
        t.start()
    for t in th:
        t.join(60.0)
    assert not any(t.is_alive() for t in th), "engine locks deadlocked"
    assert not errs, errs
    assert done[0] > 3 and done[1] > 3, done
    e.close()


def test_pipelined_stats_attribute_setup_and_pool():
    n = 1 << 18
    b = corpus.solana_txns(n, seed=32)
    e = fa.Engine(0, n, 1 << 29)
    e.dsm_pool_min = 0                     # the pooled schedule: setup on the front stream, pool on the DSM stream
    dev = torch.device("cuda", 0)
    d_blob = torch.from_numpy(np.concatenate([b.blob, np.zeros(64, np.uint8)])).to(dev)
    d_desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
    d_out = torch.zeros(n, dtype=torch.int32, device=dev)
    torch.cuda.synchronize()
    st = torch.cuda.current_stream(dev).cuda_stream
    serial = e.verify_dev_timed(n, d_blob.data_ptr(), len(b.blob), d_desc.data_ptr(), d_out.data_ptr(), st)
    e.dev_stats_begin()
    for _ in range(6):
        e.verify_dev(n, d_blob.data_ptr(), len(b.blob), d_desc.data_ptr(), d_out.data_ptr(), st, inputs_ready=True)
    torch.cuda.synchronize()
    live, launches = e.dev_stats_end()       # per-kernel mean ms over the launches
    assert launches == 6
    names = dict(zip(fa.Engine.KERNELS, range(5)))
    setup, pool = live[names["fd_k_dsm_setup"]], live[names["fd_k_dsm_pool"]]
    # setup is timed between its own front-stream events: it cannot absorb a
    # wait for the previous launch's pool (which would make it pool-sized)
    assert 0 < setup < 0.5 * pool, (live, serial)
    # the pool, from the back part's own start event, is the pool alone
    assert 0.7 * serial[names["fd_k_dsm_pool"]] < pool < 1.6 * serial[names["fd_k_dsm_pool"]], (live, serial)
    assert (live >= 0).all()
    e.close()


def test_dsm_clock_counts_pool_quad_and_oct_waves():
    """fd_ed25519_gpu_dsm_clock: every pool / quad / oct wave adds its loop's
    shader cycles and real-time ticks; the ratio is a plausible gfx950 clock
    (the bench reports it beside the roofline)"""
    e = fa.Engine(0, 1 << 18, 1 << 29)
    dev = torch.device("cuda", 0)
    st = torch.cuda.current_stream(dev).cuda_stream
    for n, pool_min in ((1 << 18, 0), (4096, 1 << 30), (64, 1 << 30)):
        b = corpus.solana_txns(n, seed=34)
        e.dsm_pool_min = pool_min
        d_blob = torch.from_numpy(np.concatenate([b.blob, np.zeros(64, np.uint8)])).to(dev)
        d_desc = torch.from_numpy(b.desc.view(np.uint8).copy()).to(dev)
        d_out = torch.zeros(n, dtype=torch.int32, device=dev)
        torch.cuda.synchronize()
        e.dsm_clock(clear=True)
        e.verify_dev(n, d_blob.data_ptr(), len(b.blob), d_desc.data_ptr(), d_out.data_ptr(), st)
        torch.cuda.synchronize()
        c = e.dsm_clock()
        assert (d_out.cpu().numpy() == 0).sum() >= n - 4
        k = "pool" if pool_min == 0 else "quad" if n > 64 else "oct"
        assert c[k]["waves"] == {"pool": n // 128, "quad": n // 16, "oct": n // 8}[k], c
        assert 1.0 < c[k]["ghz"] < 3.0, c
        for other in {"pool", "quad", "oct"} - {k}:
            assert c[other]["waves"] == 0 and c[other]["ghz"] is None, c
    e.close()


@pytest.mark.parametrize("period_ns", [0, 150_000])
def test_synth_producer_codes(ref, period_ns):
    base = corpus.adversarial_txns(20000, seed=33, invalid_frac=0.1)
    exp = oracle_batch(ref, base)
    e = fa.Engine(0, 4096, 8 << 20, depth=8)
    e.register(base.blob)
    f = fa.Feeder(e)
    starts = np.random.default_rng(3).integers(0, len(base) - 4096, 16)
    st, codes = f.synth(base.blob, base.desc, 4096, starts, 48, 6, period_ns, codes=True)
    f.close()
    e.close()
    assert (st["state"] == 1).all()
    for i in range(48):
        seg = exp[starts[i % 16]:starts[i % 16] + 4096]
        assert (codes[i] == seg).all(), i
        want = [int((seg == 0).sum()), int((seg == -1).sum()), int((seg == -2).sum()), int((seg == -3).sum()), 0]
        assert st["codes"][i].tolist() == want, i
    assert (st["t_push_ns"] <= st["t_submit_ns"]).all() and (st["t_submit_ns"] <= st["t_done_ns"]).all()
    if period_ns:
        assert (np.diff(st["t_sched_ns"].astype(np.int64)) == period_ns).all()


@pytest.mark.parametrize("cap", [1, 3, 15])
def test_tiny_engine(ref, cap):
    """Engines of a few signatures' capacity create and verify (engine
    creation warms every slot stream with copies sized to the slot's own
    buffers: the code buffer of a 1-signature engine is 4 bytes)."""
    b = corpus.adversarial(cap, 120, seed=40 + cap, invalid_frac=0.5)
    exp = oracle_batch(ref, b)
    e = fa.Engine(0, cap, 1 << 16, depth=2)
    assert (e.verify_packed(b.blob, b.desc) == exp).all()
    e.close()


def test_direct_code_write_vs_d2h_copy(ref, tmp_path):
    """ring batches of up to out_direct_max signatures have their
    codes written by the DSM straight into the slot's mapped pinned memory
    (no D2H blit), visible once the slot's done event completes.  The
    default covers the latency path (4,096); here a child process raises it
    to 65,536 and checks batches of 4,096 (quad DSM) and 40,000 (the
    uniform DSM, beyond the quad's 32,768) through the ring against the
    reference -- and against the same batches with the direct write off
    (FD_ED25519_GPU_OUT_DIRECT_MAX=0, the D2H copy)."""
    import os
    import subprocess
    import sys
    b = corpus.adversarial(40000, 110, seed=47, invalid_frac=0.2)
    exp = oracle_batch(ref, b)
    np.save(tmp_path / "exp.npy", exp)
    code = f"""
import sys, numpy as np
sys.path.insert(0, {fa.__file__.rsplit('/', 2)[0]!r})
import firedancer_amd as fa
from firedancer_amd import corpus
b = corpus.adversarial(40000, 110, seed=47, invalid_frac=0.2)
exp = np.load({str(tmp_path / 'exp.npy')!r})
e = fa.Engine(0, 40000, 1 << 24, depth=3)
for n in (4096, 40000):
    sub = corpus.Batch(b.blob, b.desc[:n])
    for rep in range(3):
        t = e.submit(sub.blob, sub.desc)
        got = np.full(n, 99, np.int32)
        assert e.poll(t, got, True)
        assert (got == exp[:n]).all(), (n, rep, int((got != exp[:n]).sum()))
e.close()
print("ok")
"""
    for od in ("65536", "0"):
        env = dict(os.environ, FD_ED25519_GPU_OUT_DIRECT_MAX=od)
        r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=240, env=env)
        assert r.returncode == 0 and r.stdout.strip().endswith("ok"), (od, r.stdout[-1000:], r.stderr[-3000:])


@pytest.mark.parametrize("depth", [1, 3])
def test_early_codes_submit_poll_back_to_back(ref, depth):
    """Round 5: a blocking poll of a direct-output batch of at most
    early_max (64) signatures returns as soon as every code has landed in
    the slot's pinned memory, before the completion event; the slot then
    retires.  Back-to-back submit -> poll on a one-slot engine must still
    find its slot (fd_wait_retiring), and every code must equal the
    reference's -- batches of 1, 17, 64 (early) and 65 (event) on the oct
    and quad DSMs, with invalid signatures mixed in."""
    b = corpus.adversarial(128, 200, seed=51, invalid_frac=0.4)
    exp = oracle_batch(ref, b)
    e = fa.Engine(0, 128, 1 << 20, depth=depth)
    for rep in range(40):
        for n in (1, 17, 64, 65):
            lo = (rep * 7) % (128 - n + 1)
            sub = corpus.Batch(b.blob, b.desc[lo:lo + n])
            t = e.submit(sub.blob, sub.desc)
            got = np.full(n, 99, np.int32)
            assert e.poll(t, got, True)
            assert (got == exp[lo:lo + n]).all(), (rep, n, lo, int((got != exp[lo:lo + n]).sum()))
    e.close()
