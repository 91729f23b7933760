"""The driver's multi-GPU bench path rehearsed on the CPU: torchrun with 2 and 4 gloo
ranks, the CPU encoder, and the per-GPU end-to-end check on every rank. Rank 0's
JSON line must carry one e2e record per rank and the node total."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [2, 4])
def test_bench_two_ranks_report_per_gpu_e2e(world, tmp_path):
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29500 + os.getpid() % 1000), "bench.py",
           "--gpus", str(world), "--backend", "cpu", "--path", "encoder", "--width", "256", "--height", "128",
           "--sessions", "1", "--steps", "3", "--warmup", "1", "--extra-4k", "0",
           "--e2e-force", "--e2e-sessions", "2", "--e2e-seconds", "2", "--e2e-warmup", "2"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    res = json.loads(line)
    assert res["n_gpus"] == world
    per = res["e2e_per_gpu"]
    assert [p["gpu"] for p in per] == list(range(world))
    assert all(p["sessions"] == 2 and p.get("error") is None for p in per), per
    if all(p["sustained"] for p in per):
        assert res["concurrent_60fps_sessions"] == 2 * world
    else:
        assert res["concurrent_60fps_sessions"] is None


def test_bench_world8_capture_path_cpu_quota(tmp_path):
    """The driver's 8-GPU command shape rehearsed with 8 gloo ranks on the CPU: the
    default capture path and the default e2e sweep (per rank 16 then 8 sessions). Each
    rank's e2e is cut to what its share of the CPU quota can drive (bench.cpu_budget:
    here 8 CPUs / 8 ranks -> no session), reported as cpu_bound with the cap, and rank 0
    still prints the node's JSON line with one record per rank."""
    world = 8
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(29700 + os.getpid() % 1000), "bench.py",
           "--gpus", str(world), "--backend", "cpu", "--width", "256", "--height", "128",
           "--sessions", "1", "--steps", "3", "--warmup", "1", "--extra-4k", "0", "--e2e-force"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-3000:]
    res = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert res["n_gpus"] == world and res["config"]["path"] == "capture"
    assert res["value"] > 0 and res["config"]["global_batch"] == world
    cpu = res["e2e_cpu"]
    assert cpu["ranks"] == world and cpu["session_cap_per_rank"] == int(max(0.0, cpu["cpus"] / world - 1.0) // 0.21)
    if cpu["session_cap_per_rank"] < 16:
        assert cpu["cpu_bound"] is True
    assert len(res["e2e_per_gpu"]) == world

