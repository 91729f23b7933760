"""Session state transfer (codec/h264_encoder.h StateHeader; parallel/migrate.py).

A session exported after frame k and imported into a fresh encoder must produce
byte-identical packets from frame k+1 on — P frames, no IDR — in-process and
across processes (gloo here; the same code moves device tensors over RCCL).
GPU variants: HIP -> HIP through a device tensor, and HIP -> CPU reference.
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from selkies_gstreamer_amd.ops.native import H264Encoder
from tests.h264_util import synthetic_frames

W, H = 160, 128
KW = dict(stripe_height=32, qp=27, paint_qp=20, paint_over_trigger=3, paint_over_burst=2)


def _frames(n=9):
    fr = list(synthetic_frames(W, H, 6, seed=8))
    return fr[:4] + [fr[3]] * 3 + fr[4:6]     # motion, static (paint-over), motion


def _run(enc, frames, start):
    return [[(p.y, p.key, p.data) for p in enc.encode(f, start + i)] for i, f in enumerate(frames)]


@pytest.mark.parametrize("num_refs", [1, 2])
@pytest.mark.parametrize("fullframe", [False, True])
def test_migrated_session_continues_bit_exact(fullframe, num_refs):
    fr = _frames()
    a = H264Encoder(W, H, fullframe=fullframe, backend="cpu", num_refs=num_refs, **KW)
    _run(a, fr[:4], 0)
    a.set_qp(30, 19)
    state = a.export_state()
    b = H264Encoder(W, H, fullframe=fullframe, backend="cpu", num_refs=num_refs, **KW)
    b.import_state(state)
    ra, rb = _run(a, fr[4:], 4), _run(b, fr[4:], 4)
    assert ra == rb
    assert not any(key for frame in rb for _, key, _ in frame)      # no IDR after the move
    fresh = H264Encoder(W, H, fullframe=fullframe, backend="cpu", num_refs=num_refs, **KW)
    assert any(key for _, key, _ in _run(fresh, fr[4:5], 4)[0])     # without state: IDR


def test_state_geometry_is_checked():
    a = H264Encoder(W, H, backend="cpu", **KW)
    b = H264Encoder(W, H + 32, backend="cpu", **KW)
    s = a.export_state()
    with pytest.raises(RuntimeError, match="geometry"):
        b.import_state(np.resize(s, b.state_bytes()))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, port, q):
    import torch.distributed as dist
    from selkies_gstreamer_amd.parallel import fanout, migrate
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    fr = _frames()
    enc = H264Encoder(W, H, backend="cpu", **KW)
    if rank == 0:
        _run(enc, fr[:5], 0)
        migrate.send_session(enc, 1)
        out = _run(enc, fr[5:], 5)
    else:
        migrate.recv_session(enc, 0)
        out = _run(enc, fr[5:], 5)
    both = fanout.broadcast_object(out, src=1) if rank == 0 else fanout.broadcast_object(out, src=1)
    if rank == 0:
        q.put(out == both)
    dist.destroy_process_group()


def test_session_moves_between_processes():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, port, q)) for r in range(2)]
    for p in ps:
        p.start()
    for p in ps:
        p.join(120)
    assert all(p.exitcode == 0 for p in ps)
    assert q.get(timeout=5) is True


@pytest.mark.gpu
def test_hip_session_moves_through_device_tensor_and_to_cpu():
    from selkies_gstreamer_amd.parallel import migrate
    fr = _frames()
    a = H264Encoder(W, H, backend="hip", **KW)
    _run(a, fr[:4], 0)
    t = migrate.export_tensor(a)                       # device tensor (what RCCL would carry)
    assert t.is_cuda
    b = H264Encoder(W, H, backend="hip", **KW)
    migrate.import_tensor(b, t)
    c = H264Encoder(W, H, backend="cpu", **KW)
    c.import_state(a.export_state())                   # host snapshot -> CPU reference
    ra, rb, rc = _run(a, fr[4:], 4), _run(b, fr[4:], 4), _run(c, fr[4:], 4)
    assert ra == rb == rc
    assert not any(key for frame in rb for _, key, _ in frame)


@pytest.mark.parametrize("codec", ["hevc", "av1"])
@pytest.mark.parametrize("rc", ["crf", "cbr"])
def test_migrated_hevc_av1_session_continues_bit_exact(codec, rc):
    """HEVC and AV1 sessions migrate like H.264 ones (StateHeader v3: controller, K10
    rate-control state and the filtered reference): the importing encoder codes the
    next frames as inter frames, byte-identical to the session that never moved, so the
    client's decoder continues without a key frame."""
    fr = _frames()
    kw = dict(codec=codec, fullframe=True, backend="cpu", qp=27, rate_control=rc, bitrate_kbps=600 if rc == "cbr" else 0)
    a = H264Encoder(W, H, **kw)
    _run(a, fr[:4], 0)
    state = a.export_state()
    b = H264Encoder(W, H, **kw)
    b.import_state(state)
    ra, rb = _run(a, fr[4:], 4), _run(b, fr[4:], 4)
    assert ra == rb
    assert not any(key for frame in rb for _, key, _ in frame)
    assert a.rc_stats() == b.rc_stats()
    with pytest.raises(RuntimeError, match="codec"):
        H264Encoder(W, H, codec="av1" if codec == "hevc" else "hevc", fullframe=True, backend="cpu").import_state(state)


def _worker_codec(rank, port, q, codec):
    import torch.distributed as dist
    from selkies_gstreamer_amd.parallel import fanout, migrate
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=2)
    fr = _frames()
    enc = H264Encoder(W, H, codec=codec, fullframe=True, backend="cpu", qp=27)
    if rank == 0:
        _run(enc, fr[:5], 0)
        migrate.send_session(enc, 1)
        out = _run(enc, fr[5:], 5)
    else:
        migrate.recv_session(enc, 0)
        out = _run(enc, fr[5:], 5)
    both = fanout.broadcast_object(out, src=1)
    if rank == 0:
        q.put(out == both and not any(key for frame in both for _, key, _ in frame))
    dist.destroy_process_group()


@pytest.mark.parametrize("codec", ["hevc", "av1"])
def test_hevc_av1_session_moves_between_processes(codec):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_codec, args=(r, port, q, codec)) for r in range(2)]
    for p in ps:
        p.start()
    ok = q.get(timeout=300)
    for p in ps:
        p.join(timeout=120)
    assert ok


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["hevc", "av1"])
def test_hip_hevc_av1_session_moves_through_device_tensor_and_to_cpu(codec):
    """HIP -> HIP (device tensor, the buffer RCCL carries) and HIP -> CPU reference for
    the HEVC and AV1 back ends (CBR: the K10 state travels too)."""
    from selkies_gstreamer_amd.parallel import migrate
    fr = _frames()
    kw = dict(codec=codec, fullframe=True, qp=27, rate_control="cbr", bitrate_kbps=600)
    a = H264Encoder(W, H, backend="hip", **kw)
    _run(a, fr[:4], 0)
    t = migrate.export_tensor(a)
    assert t.is_cuda
    b = H264Encoder(W, H, backend="hip", **kw)
    migrate.import_tensor(b, t)
    c = H264Encoder(W, H, backend="cpu", **kw)
    c.import_state(a.export_state())
    ra, rb, rc = _run(a, fr[4:], 4), _run(b, fr[4:], 4), _run(c, fr[4:], 4)
    assert ra == rb == rc
    assert not any(key for frame in rb for _, key, _ in frame)


def _worker_hip(rank, port, q, codec):
    import torch.distributed as dist
    from selkies_gstreamer_amd.parallel import fanout, migrate
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    # two processes on the box's one GPU: gloo carries the device state through host
    # memory (RCCL refuses two ranks on one device); on a node it is RCCL over xGMI
    dist.init_process_group("gloo", rank=rank, world_size=2)
    fr = _frames()
    kw = dict(codec=codec, fullframe=codec != "h264", qp=27, rate_control="cbr", bitrate_kbps=600)
    enc = H264Encoder(W, H, backend="hip", **kw)
    if rank == 0:
        _run(enc, fr[:5], 0)
        migrate.send_session(enc, 1)
    else:
        migrate.recv_session(enc, 0)
    out = _run(enc, fr[5:], 5)
    both = fanout.broadcast_object(out, src=1)
    if rank == 0:
        q.put(out == both and not any(key for frame in both for _, key, _ in frame))
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("codec", ["h264", "hevc", "av1"])
def test_hip_session_moves_between_processes_on_one_gpu(codec):
    """Two processes on one GPU: rank 0's HIP session continues in rank 1's encoder with
    P frames, byte-identical to rank 0 continuing it."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker_hip, args=(r, port, q, codec)) for r in range(2)]
    for p in ps:
        p.start()
    ok = q.get(timeout=100)
    for p in ps:
        p.join(timeout=60)
    assert ok
