"""One session across ranks (parallel/dist_banded.py): bands scattered from rank 0,
encoded per rank, packets gathered back — gloo + CPU encoder here (the RCCL/HIP path
is the same code with cuda tensors). The packets must equal those of one encoder of
the whole frame, keyframe requests from rank 0 must reach every band, and QP changes
must apply everywhere."""
import os
import socket

import pytest


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_dir, W, H, sh):
    import torch.distributed as dist
    from selkies_gstreamer_amd.ops.native import H264Encoder
    from selkies_gstreamer_amd.parallel.dist_banded import DistBandedEncoder
    from tests.h264_util import synthetic_frames
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    enc = DistBandedEncoder(W, H, stripe_height=sh, backend="cpu", qp=27)
    ref = H264Encoder(W, H, stripe_height=sh, backend="cpu", qp=27) if rank == 0 else None
    frames = synthetic_frames(W, H, 6, seed=5)
    ok = True
    for t, f in enumerate(frames):
        if rank == 0 and t == 3:
            enc.request_keyframe()
            ref.request_keyframe()
        if rank == 0 and t == 4:
            enc.set_qp(33)
            ref.set_qp(33)
        got = enc.encode(f if rank == 0 else None, t)
        if rank == 0:
            want = ref.encode(f, t)
            ok &= sorted((p.y, p.data, p.key) for p in got) == sorted((p.y, p.data, p.key) for p in want)
            if t == 3:
                ok &= len(got) == (H + sh - 1) // sh and all(p.key for p in got)
        else:
            ok &= got is None
    enc.close()
    if rank == 0:
        with open(os.path.join(out_dir, "result.txt"), "w") as fh:
            fh.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


@pytest.mark.parametrize("world,W,H,sh", [(2, 160, 200, 32), (3, 128, 192, 32), (4, 128, 256, 32)])
def test_dist_banded_matches_single_encoder(tmp_path, world, W, H, sh):
    import torch.multiprocessing as mp
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path), W, H, sh), nprocs=world, join=True)
    assert (tmp_path / "result.txt").read_text() == "ok"


def test_pack_roundtrip():
    from selkies_gstreamer_amd.ops.native import Packet
    from selkies_gstreamer_amd.parallel.dist_banded import _pack, _unpack
    pk = [Packet(b"\x04abc", 64, 1920, 64, True), Packet(b"", 0, 8, 16, False)]
    assert _unpack(_pack(pk)) == pk


@pytest.mark.gpu
def test_upload_ptr_from_device_memory_matches_host_upload():
    import torch
    from selkies_gstreamer_amd.ops.native import H264Encoder
    from tests.h264_util import synthetic_frames
    W, H = 320, 192
    a = H264Encoder(W, H, stripe_height=64, backend="hip", qp=27)
    b = H264Encoder(W, H, stripe_height=64, backend="hip", qp=27)
    try:
        for t, f in enumerate(synthetic_frames(W, H, 4, seed=2)):
            want = a.encode(f, t)
            dev = torch.from_numpy(f).cuda()
            torch.cuda.synchronize()
            b.upload_ptr(dev.data_ptr(), W * 4, t, keepalive=dev)
            b.launch()
            got = b.finish()
            assert [(p.y, p.data) for p in got] == [(p.y, p.data) for p in want]
    finally:
        a.close()
        b.close()


def _nccl_worker(rank, world, port, out_dir):
    import torch
    import torch.distributed as dist
    from selkies_gstreamer_amd.ops.native import H264Encoder
    from selkies_gstreamer_amd.parallel.dist_banded import DistBandedEncoder
    from tests.h264_util import synthetic_frames
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world,
                            device_id=torch.device("cuda", 0))
    W, H = 320, 256
    enc = DistBandedEncoder(W, H, stripe_height=64, backend="hip", qp=27)
    ref = H264Encoder(W, H, stripe_height=64, backend="hip", qp=27)
    ok = True
    for t, f in enumerate(synthetic_frames(W, H, 4, seed=3)):
        got = enc.encode(torch.from_numpy(f).cuda(), t)
        want = ref.encode(f, t)
        ok &= sorted((p.y, p.data) for p in got) == sorted((p.y, p.data) for p in want)
    enc.close()
    ref.close()
    with open(os.path.join(out_dir, "result.txt"), "w") as fh:
        fh.write("ok" if ok else "mismatch")
    dist.destroy_process_group()


@pytest.mark.gpu
def test_dist_banded_rccl_single_rank(tmp_path):
    """The RCCL path (scatter from device memory, D2D upload, all_gather of packets) on
    one GPU; more ranks need more GPUs (the driver's multi-GPU node)."""
    import torch.multiprocessing as mp
    mp.spawn(_nccl_worker, args=(1, _free_port(), str(tmp_path)), nprocs=1, join=True)
    assert (tmp_path / "result.txt").read_text() == "ok"
