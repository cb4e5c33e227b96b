"""bench.py's own N-rank code path on the CPU (gloo, world size 2): the
torch.distributed.run launch the driver uses, the barrier-bracketed timed
region, the max-over-ranks wall time and the whole-job aggregate
(value = sigs per step x steps x ranks / max elapsed), with a fixed host
step standing in for the GPU launch (--dry-cpu)."""
import json
import os
import socket
import subprocess
import sys

from conftest import ROOT


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_gloo():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "5", "--warmup", "2", "--dry-cpu"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [x for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout                 # rank 0 prints ONE line
    res = json.loads(lines[0])
    assert res["n_gpus"] == 2 and res["steps"] == 5 and res["warmup"] == 2
    assert res["scaling"] == "weak" and res["higher_is_better"] is True
    n_step = res["config"]["sigs_per_step_per_gpu"]
    elapsed = res["ms_per_step"] * res["steps"] / 1e3
    assert abs(res["value"] - n_step * 5 * 2 / elapsed) / res["value"] < 1e-6
    assert "not a measurement" in res["data"]


def test_bench_single_rank_dry():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "3", "--warmup", "1", "--dry-cpu"],
                       capture_output=True, text=True, timeout=120, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    res = json.loads(r.stdout.strip().splitlines()[-1])
    assert res["n_gpus"] == 1 and res["value"] > 0


def test_traffic_summary_held_to_the_kernels_build(tmp_path):
    """roofline.traffic only from a PMC summary of the loaded device code
    (fd_ed25519_gpu_kernels_id) at this launch size; the committed summary
    must be of the committed kernels"""
    sys.path.insert(0, ROOT)
    import bench
    import firedancer_amd as fa
    kid = fa.kernels_id()
    assert len(kid) == 16 and kid != "unknown"
    p = tmp_path / "t.json"
    p.write_text(json.dumps({"kernels_id": kid, "sigs_per_launch": 1024,
                             "kernels": {"fd_k_dsm_pool": {"hbm_bytes_per_launch": 5.0}}}))
    assert bench.load_traffic(str(p), 1024, "fd_k_dsm_pool", kid) == (5.0, "current")
    v, st = bench.load_traffic(str(p), 1024, "fd_k_dsm_pool", "0" * 16)
    assert v is None and st.startswith("stale")
    v, st = bench.load_traffic(str(p), 2048, "fd_k_dsm_pool", kid)
    assert v is None
    committed = json.load(open(os.path.join(ROOT, "profiles", "pmc_traffic.json")))
    assert committed.get("kernels_id") == kid, "profiles/pmc_traffic.json is not of these kernels: rerun tools/gpu.sh pmcthr"
