"""Session placement, node launcher supervision, and packet fan-in over
torch.distributed (gloo, world_size 2, CPU encoders) — the multi-GPU paths
exercised without GPUs."""
import asyncio
import os
import socket
import sys

import pytest

from selkies_gstreamer_amd.parallel.launcher import SessionSpec, Supervisor, plan_sessions
from selkies_gstreamer_amd.parallel.placement import SessionPlacer, session_weight


def test_placement_least_loaded_and_capacity():
    p = SessionPlacer(2, capacity_per_gpu=2.0)
    assert [p.acquire(f"s{i}") for i in range(4)] == [0, 1, 0, 1]
    assert p.acquire("s4") is None                      # node full
    p.release("s1")
    assert p.acquire("s5") == 1
    assert p.acquire("s5") == 1                         # idempotent
    p.update_external_load({0: 0.9})
    p.release("s0")
    p.release("s2")
    p.release("s3")
    p.release("s5")
    assert p.acquire("x") == 1                          # GPU 0 is busy with foreign work
    assert session_weight(3840, 2160, 60) == pytest.approx(4.0)
    snap = p.snapshot()
    assert snap[1]["sessions"] == ["x"]


def test_plan_sessions():
    specs = plan_sessions(4, 2, 9000, 30, extra=["--capture-source", "synthetic"])
    assert [(s.display, s.port, s.gpu) for s in specs] == [(":30", 9000, 0), (":31", 9001, 1), (":32", 9002, 0),
                                                           (":33", 9003, 1)]
    cmd = specs[0].command("python")
    assert cmd[:3] == ["python", "-m", "selkies_gstreamer_amd"] and "--gpu-id" in cmd and cmd[-1] == "synthetic"
    assert specs[1].env({})["DISPLAY"] == ":31"
    with pytest.raises(RuntimeError):
        plan_sessions(5, 1, 9000, 30, capacity=4)
    assert "GPU_MAX_HW_QUEUES" not in specs[0].env({})  # 2 sessions per GPU: HIP's default queues
    dense = plan_sessions(12, 1, 9000, 30)
    assert dense[0].env({})["GPU_MAX_HW_QUEUES"] == "2"
    assert dense[0].env({"GPU_MAX_HW_QUEUES": "1"})["GPU_MAX_HW_QUEUES"] == "1"  # operator's choice wins


class _Crashing(SessionSpec):
    def command(self, python=sys.executable):
        return [python, "-c", "import sys; sys.exit(3)"]


def test_supervisor_restarts_failed_sessions():
    async def main():
        sup = Supervisor([_Crashing("a", ":99", 1, 0)], health_interval=0.1, max_backoff=0.2, check_health=False)
        task = asyncio.create_task(sup.run())
        await asyncio.sleep(2.0)
        await sup.stop()
        task.cancel()
        return sup.restarts["a"]
    assert asyncio.run(main()) >= 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir):
    import torch.distributed as dist
    from selkies_gstreamer_amd.ops.native import H264Encoder
    from selkies_gstreamer_amd.parallel.fanout import broadcast_object, gather_packets
    from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    key = broadcast_object({"keyframe": True} if rank == 0 else None)
    src = SyntheticDesktop(96, 64, kind="motion", seed=rank)
    enc = H264Encoder(96, 64, stripe_height=32, backend="cpu")
    total = 0
    for t in range(3):
        pk = enc.encode(src.frame(t), t)
        got = gather_packets([(rank * 10 + i, p.data) for i, p in enumerate(pk)])
        if rank == 0:
            total += len(got)
            assert {r for r, _, _ in got} == set(range(world))
            assert all(d[0] == 0x04 for _, _, d in got)
        else:
            assert got is None
    if rank == 0:
        with open(os.path.join(out_dir, "result.txt"), "w") as f:
            f.write(f"{total} {key['keyframe']}")
    dist.destroy_process_group()


def test_gather_packets_gloo_world2(tmp_path):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path)), nprocs=2, join=True)
    total, key = (tmp_path / "result.txt").read_text().split()
    assert int(total) >= 2 * 2 * 3 and key == "True"   # 2 stripes x 2 ranks x 3 frames (motion)
