"""Session migration and hot-standby replicas over torch.distributed.

A streaming session's inter-frame state — reference picture(s), the damage
baseline (last source), the MV field, the stripe controller (frame_num /
idr_pic_id / paint-over counters per stripe) and the K10 rate-control state — is
exported as one flat buffer (codec/h264_encoder.h ``StateHeader`` v3 layout, the
same for the CPU and HIP backends of all three codecs: H.264, HEVC and AV1; the
header names the codec and an import into another codec's encoder is refused). For a HIP encoder the buffer is a device tensor, so moving a session
to another GPU of the node is one point-to-point transfer over xGMI (RCCL send /
recv, or a broadcast to every GPU for standby replicas), and the new GPU codes
its next frame as a P frame against the migrated reference: the clients' stripe
decoders never see an IDR (what the reference can only do by restarting the
pipeline and forcing a keyframe).

1080p state is ~6.3 MB (two 4:2:0 planes sets + MV field): ~40 µs on one xGMI link.

Inside one server process the same state moves a running display between GPUs
(csrc/runtime/capture.cpp ``CaptureSession::move_to``, driven by
parallel/rebalance.py); this module is the cross-process path. Over a ``gloo``
group device tensors travel through host memory (gloo carries CPU tensors).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from ..ops.native import H264Encoder


def _device_of(enc: H264Encoder) -> torch.device:
    if enc.backend == "hip":
        return torch.device("cuda", enc.cfg.device)
    return torch.device("cpu")


def state_tensor(enc: H264Encoder) -> torch.Tensor:
    """An uninitialised uint8 tensor of the encoder's state size on its device."""
    return torch.empty(enc.state_bytes(), dtype=torch.uint8, device=_device_of(enc))


def export_tensor(enc: H264Encoder) -> torch.Tensor:
    t = state_tensor(enc)
    if t.is_cuda:
        torch.cuda.synchronize(t.device)
    enc.export_state(t)
    return t


def import_tensor(enc: H264Encoder, t: torch.Tensor) -> None:
    if t.is_cuda:
        torch.cuda.synchronize(t.device)
    if t.device != _device_of(enc):
        t = t.to(_device_of(enc))
    enc.import_state(t)


def _wire(t: torch.Tensor, group) -> torch.Tensor:
    """The tensor the group's backend can carry: gloo moves host tensors only."""
    return t.cpu() if t.is_cuda and dist.get_backend(group) == "gloo" else t


def send_session(enc: H264Encoder, dst: int, group=None) -> None:
    """Sends the session state to rank ``dst`` (RCCL over xGMI for GPU encoders)."""
    dist.send(_wire(export_tensor(enc), group), dst, group=group)


def recv_session(enc: H264Encoder, src: int, group=None) -> None:
    """Receives a session state from rank ``src`` into ``enc`` (same geometry/config)."""
    t = _wire(state_tensor(enc), group)
    dist.recv(t, src, group=group)
    import_tensor(enc, t)


def broadcast_session(enc: H264Encoder, src: int, group=None) -> None:
    """Every rank's ``enc`` ends up with rank ``src``'s session state (standby replicas)."""
    t = _wire(export_tensor(enc) if dist.get_rank(group) == src else state_tensor(enc), group)
    dist.broadcast(t, src, group=group)
    if dist.get_rank(group) != src:
        import_tensor(enc, t)
