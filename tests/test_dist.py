"""bench.py's multi-rank path (one process per GPU, gloo barrier + max-over-ranks)
exercised on CPU with world_size 2 and a stub registration (--selftest)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_bench_two_ranks_gloo(tmp_path):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", OMP_NUM_THREADS="1")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", "--master-port=29531", os.path.join(ROOT, "bench.py"),
           "--gpus", "2", "--steps", "5", "--warmup", "1", "--config", "c2", "--selftest"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout  # rank 0 only
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["steps"] == 5 and d["warmup"] == 1 and d["scaling"] == "weak"
    # value = K summed over both ranks / the slowest rank's wall time
    assert abs(d["value"] - 2 * 5 * 100 / (d["ms_per_step"] * 5 / 1e3)) / d["value"] < 1e-6
    assert d["data"] == "selftest-stub" and "cpu_baseline" not in d
    # the strong-scaling leg: one child process per rank, results merged by rank 0
    sh = d["sharded"]
    assert set(sh) == {"c4", "c5"} and sh["c4"]["ranks"] == 2 and sh["c5"]["ranks"] == 2, sh
    assert sh["c5"]["ms_per_registration"] == 5 * 0.001 / 5 * 1e3 and sh["c5"]["speedup_vs_one_gpu"] == 2.0


def test_bench_gpus2_self_launch(tmp_path):
    """--gpus 2 with no external launcher: bench.py starts its own two rank processes
    and reports n_gpus 2 (never silently one GPU)."""
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["OMP_NUM_THREADS"] = "1"
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "4", "--warmup", "1",
           "--config", "c2", "--selftest"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = json.loads(lines[0])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"] == "replicas x2"
    assert abs(d["value"] - 2 * 4 * 100 / (d["ms_per_step"] * 4 / 1e3)) / d["value"] < 1e-6


def test_bench_world_size_mismatch_fails(tmp_path):
    env = dict(os.environ, WORLD_SIZE="1", RANK="0", LOCAL_RANK="0")
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "1", "--warmup", "0",
           "--config", "c2", "--selftest"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=120, env=env, cwd=str(tmp_path))
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
