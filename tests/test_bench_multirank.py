"""bench.py's multi-rank path (barrier, MAX/SUM reductions, rank-0 JSON, packet
gather) rehearsed on the CPU backend with gloo and two ranks — the same code the
driver runs with RCCL on 1/2/4/8 MI355X."""
import json
import socket
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_cpu_bench():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
           "--backend", "cpu", "--gpus", "2", "--steps", "2", "--warmup", "1", "--sessions", "2",
           "--width", "256", "--height", "128", "--pool", "2", "--gather", "--path", "encoder"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout              # rank 0 only
    d = lines[0]
    assert d["n_gpus"] == 2 and d["steps"] == 2 and d["scaling"] == "weak"
    assert d["config"]["global_batch"] == 4
    assert abs(d["value"] - 8 / (d["ms_per_step"] * 2 / 1e3)) / d["value"] < 0.05   # 2 ranks x 2 sessions x 2 steps
    assert d["gathered_bytes_rank0"] > 0


def test_two_rank_cpu_dist_bands():
    """--dist-bands: one session split across the ranks (strong scaling JSON)."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
           "--backend", "cpu", "--gpus", "2", "--steps", "2", "--warmup", "1",
           "--width", "256", "--height", "256", "--pool", "2", "--dist-bands"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = lines[0]
    assert d["n_gpus"] == 2 and d["scaling"] == "strong" and d["config"]["bands"] == [[0, 128], [128, 256]]
    assert d["kib_per_frame"] > 0


def test_two_rank_cpu_bench_default_capture_path():
    """The driver's N>1 command shape (default --path capture, no --gather) on gloo."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_port()), str(ROOT / "bench.py"),
           "--backend", "cpu", "--gpus", "2", "--steps", "2", "--warmup", "1", "--sessions", "2",
           "--width", "256", "--height", "128", "--pool", "2"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1 and lines[0]["n_gpus"] == 2 and lines[0]["config"]["path"] == "capture"
