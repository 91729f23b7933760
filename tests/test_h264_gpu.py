"""HIP (gfx950) H.264 pipeline: bit-exact against the CPU reference encoder and
decodable by the independent verification decoder."""
import numpy as np
import pytest

from selkies_gstreamer_amd.ops.native import H264Encoder, MB_INFO_DTYPE, ME_DTYPE, TASK_DTYPE
from selkies_gstreamer_amd.utils.synthetic import SyntheticDesktop
from tests.h264_util import StripeDecoder, synthetic_frames, bgrx_to_y709, psnr

pytestmark = pytest.mark.gpu


def _pair(W, H, **kw):
    return H264Encoder(W, H, backend="cpu", **kw), H264Encoder(W, H, backend="hip", **kw)


def _compare_state(cpu, gpu, W, t):
    for name in ("src_y", "src_u", "src_v"):
        a, b = cpu.debug_buffer(name), gpu.debug_buffer(name)
        assert np.array_equal(a, b), f"frame {t}: {name} differs ({np.sum(a != b)} bytes)"
    ta, tb = cpu.debug_buffer("tasks", TASK_DTYPE), gpu.debug_buffer("tasks", TASK_DTYPE)
    assert np.array_equal(ta["final_action"], tb["final_action"]), f"frame {t}: slice decisions differ"
    # per-MB decisions of every coded slice: MVs, MVDs, reference, type, modes, QP, CBP, nnz
    mb_w = (W + 15) // 16
    ia, ib = cpu.debug_buffer("mbs", MB_INFO_DTYPE), gpu.debug_buffer("mbs", MB_INFO_DTYPE)
    ma, mb = cpu.debug_buffer("me", ME_DTYPE), gpu.debug_buffer("me", ME_DTYPE)
    for task in ta:
        if task["final_action"] not in (1, 2):   # ACT_P / ACT_I (none / skip-all code no MBs)
            continue
        sl = slice(task["first_row"] * mb_w, (task["first_row"] + task["num_rows"]) * mb_w)
        for f in ("type", "mvx", "mvy", "mvdx", "mvdy", "ref", "i16_mode", "chroma_mode", "qp", "cbp", "nnz"):
            assert np.array_equal(ia[f][sl], ib[f][sl]), f"frame {t}: MB {f} differs in rows from {task['first_row']}"
        if task["final_action"] == 1:   # P slice: the motion search result it was coded from
            for f in ("mvx", "mvy", "ref"):
                assert np.array_equal(ma[f][sl], mb[f][sl]), f"frame {t}: ME {f} differs"
    for name in ("ref_y", "ref_u", "ref_v"):
        a, b = cpu.debug_buffer(name), gpu.debug_buffer(name)
        assert np.array_equal(a, b), f"frame {t}: {name} differs ({np.sum(a != b)} bytes)"


@pytest.mark.parametrize("num_refs", [1, 2])
@pytest.mark.parametrize("deblock", [False, True])
@pytest.mark.parametrize("fullframe", [False, True])
@pytest.mark.parametrize("kind", ["desktop", "noise"])
def test_gpu_matches_cpu_reference(fullframe, kind, deblock, num_refs):
    W, H = 192, 128
    cpu, gpu = _pair(W, H, stripe_height=32, fullframe=fullframe, qp=26, deblock=deblock, num_refs=num_refs)
    sd = StripeDecoder(W, H)
    for t, f in enumerate(synthetic_frames(W, H, 6, seed=3, kind=kind)):
        pc = cpu.encode(f, t)
        pg = gpu.encode(f, t)
        _compare_state(cpu, gpu, W, t)
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}: bitstreams differ"
        for p in pg:
            sd.feed(p.data)
        assert psnr(sd.Y, bgrx_to_y709(f)) > 30


@pytest.mark.parametrize("fullframe", [False, True])
def test_gpu_auto_deblock_cbr_matches_cpu(fullframe):
    """deblock='auto' under a tight CBR: the controller's dithered slice QPs straddle 34,
    so some stripes of a frame are deblocked and others not (per-slice idc); the GPU
    (k_commit / k_deblock_* gated per slice) equals the CPU reference, and the decoder
    reproduces the reference."""
    W, H = 320, 192
    kw = dict(stripe_height=32, fullframe=fullframe, deblock="auto", rate_control="cbr", bitrate_kbps=2500,
              use_paint_over=False)
    cpu, gpu = _pair(W, H, **kw)
    sd = StripeDecoder(W, H)
    src = SyntheticDesktop(W, H, kind="motion")
    qps = set()
    for t in range(40):
        f = src.frame(t)
        pc = cpu.encode(f, t)
        pg = gpu.encode(f, t)
        _compare_state(cpu, gpu, W, t)
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}: bitstreams differ"
        for p in pg:
            sd.feed(p.data)
        ref = gpu.debug_buffer("ref_y").reshape(-1, (W + 15) // 16 * 16)[:H, :W]
        assert np.array_equal(sd.Y, ref), f"frame {t}: decoder != reference"
        tk = cpu.debug_buffer("tasks", TASK_DTYPE)
        qps |= {int(q) for a, q in zip(tk["final_action"], tk["qp"]) if a in (1, 2)}
    assert min(qps) < 34 <= max(qps), qps   # both kinds of slices occurred


@pytest.mark.parametrize("deblock", [False, True])
def test_gpu_1080p_desktop_matches_cpu(deblock):
    W, H = 1920, 1080
    cpu, gpu = _pair(W, H, stripe_height=64, qp=25, deblock=deblock)
    for t, f in enumerate(synthetic_frames(W, H, 3, seed=5)):
        pc = cpu.encode(f, t)
        pg = gpu.encode(f, t)
        _compare_state(cpu, gpu, W, t)
        assert len(pc) == len(pg)
        for a, b in zip(pc, pg):
            assert a.data == b.data, f"frame {t} stripe y={a.y} differs"


def test_gpu_1080p_motion_long_matches_cpu():
    """20 frames of the bench's moving desktop through a 16-frame pool (the wrap is a
    scene cut: I stripes inside P frames), state and MVs compared every frame."""
    W, H = 1920, 1080
    cpu, gpu = _pair(W, H, stripe_height=64, qp=25)
    src = SyntheticDesktop(W, H, kind="motion")
    pool = [src.frame(i) for i in range(16)]
    for t in range(20):
        f = pool[t % 16]
        pc = cpu.encode(f, t)
        pg = gpu.encode(f, t)
        _compare_state(cpu, gpu, W, t)
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}: bitstreams differ"


def test_gpu_escalation_and_odd_geometry():
    W, H = 130, 70
    cpu, gpu = _pair(W, H, stripe_height=48, qp=4, paint_qp=4)
    for t, f in enumerate(synthetic_frames(W, H, 3, seed=9, kind="noise")):
        assert [p.data for p in gpu.encode(f, t)] == [p.data for p in cpu.encode(f, t)]
    m = gpu.debug_buffer("mbs", MB_INFO_DTYPE)
    assert m["qp"].max() > 4


@pytest.mark.parametrize("fullframe", [False, True])
def test_gpu_controller_matches_cpu(fullframe):
    """Stripe controller on the GPU (k_plan): damage streaks, paint-over bursts,
    keyframe requests and frame_num/idr_pic_id bookkeeping match the host controller."""
    W, H = 160, 96
    kw = dict(stripe_height=32, fullframe=fullframe, qp=28, paint_qp=20, paint_over_trigger=3,
              paint_over_burst=2, damage_threshold=2, damage_duration=3)
    cpu, gpu = _pair(W, H, **kw)
    moving = list(synthetic_frames(W, H, 5, seed=11))
    seq = moving[:4] + [moving[3]] * 8 + [moving[4]] * 6
    for t, f in enumerate(seq):
        if t in (7, 15):
            cpu.request_keyframe()
            gpu.request_keyframe()
        pc, pg = cpu.encode(f, t), gpu.encode(f, t)
        ta, tb = cpu.debug_buffer("tasks", TASK_DTYPE), gpu.debug_buffer("tasks", TASK_DTYPE)
        assert np.array_equal(ta, tb), f"frame {t}: slice plans differ"
        assert [(p.y, p.key, p.data) for p in pg] == [(p.y, p.key, p.data) for p in pc], f"frame {t}"


def test_gpu_overlapped_upload_matches_sequential():
    """upload(n+1) while frame n encodes, then finish(n) / launch(n+1): same packets
    as plain encode() (double-buffered input, frame id read at launch)."""
    W, H = 320, 192
    frames = list(synthetic_frames(W, H, 6, seed=12))
    a = H264Encoder(W, H, stripe_height=64, qp=26, backend="hip")
    b = H264Encoder(W, H, stripe_height=64, qp=26, backend="hip")
    ref = [[p.data for p in a.encode(f, t)] for t, f in enumerate(frames)]
    got = []
    b.upload(frames[0], 0)
    b.launch()
    for t in range(len(frames)):
        if t + 1 < len(frames):
            b.upload(frames[t + 1], t + 1)
        got.append([p.data for p in b.finish()])
        if t + 1 < len(frames):
            b.launch()
    assert got == ref


@pytest.mark.parametrize("fullframe", [False, True])
def test_gpu_two_references_toggling_matches_cpu(fullframe):
    """Second reference picture (sliding-window DPB): caret/button toggles coded as
    ref_idx 1 copies; HIP bitstreams == CPU reference, ref1 planes identical."""
    from tests.test_h264_cpu import _toggle_frames
    W, H = 160, 96
    kw = dict(stripe_height=32, fullframe=fullframe, qp=24, use_paint_over=False, num_refs=2, deblock=True)
    cpu, gpu = _pair(W, H, **kw)
    for t, f in enumerate(_toggle_frames(W, H, 8)):
        assert [p.data for p in gpu.encode(f, t)] == [p.data for p in cpu.encode(f, t)], f"frame {t}"
        assert np.array_equal(gpu.debug_buffer("ref1_y"), cpu.debug_buffer("ref1_y")), f"frame {t}"


def _two_in_flight(enc, frames, key_at=None):
    """upload(n+1) + launch(n+1) before finish(n): two frames in flight."""
    got = []
    enc.upload(frames[0], 0)
    enc.launch()
    for t in range(len(frames)):
        if t + 1 < len(frames):
            if key_at == t + 1:
                enc.request_keyframe()
            enc.upload(frames[t + 1], t + 1)
            enc.launch()
        got.append([(p.y, p.key, p.data) for p in enc.finish()])
    return got


@pytest.mark.parametrize("fullframe", [False, True])
def test_gpu_two_frames_in_flight_match_cpu(fullframe):
    """Per-parity host outputs (packets, slice decisions, frame id): with frame n+1
    launched before frame n is collected, every frame's packets equal the CPU
    reference's, including a keyframe requested mid-stream."""
    W, H = 320, 192
    frames = list(synthetic_frames(W, H, 8, seed=21))
    cpu = H264Encoder(W, H, stripe_height=64, qp=26, backend="cpu", fullframe=fullframe)
    ref = []
    for t, f in enumerate(frames):
        if t == 5:
            cpu.request_keyframe()
        ref.append([(p.y, p.key, p.data) for p in cpu.encode(f, t)])
    gpu = H264Encoder(W, H, stripe_height=64, qp=26, backend="hip", fullframe=fullframe)
    assert _two_in_flight(gpu, frames, key_at=5) == ref


@pytest.mark.parametrize("fullframe", [False, True])
@pytest.mark.parametrize("kind", ["desktop", "noise"])
def test_gpu_aq_matches_cpu(fullframe, kind):
    """MB-level adaptive QP (k_aq + start QPs in k_code_inter / k_intra_prep): per-MB
    offsets, QPs and bitstreams identical to the CPU reference; offsets really vary."""
    W, H = 256, 160
    cpu, gpu = _pair(W, H, stripe_height=32, fullframe=fullframe, qp=26, aq_strength=1.0)
    sd = StripeDecoder(W, H)
    for t, f in enumerate(synthetic_frames(W, H, 5, seed=11, kind=kind)):
        pc, pg = cpu.encode(f, t), gpu.encode(f, t)
        ta = cpu.debug_buffer("tasks", TASK_DTYPE)
        qa = np.frombuffer(cpu.debug_buffer("aq", np.uint8), np.int8).reshape(-1, (W + 15) // 16)
        qg = np.frombuffer(gpu.debug_buffer("aq", np.uint8), np.int8).reshape(-1, (W + 15) // 16)
        for task in ta:
            if task["final_action"] in (1, 2):   # offsets only exist for coded slices
                rows = slice(task["first_row"], task["first_row"] + task["num_rows"])
                assert np.array_equal(qa[rows], qg[rows]), f"frame {t}: AQ offsets differ"
        _compare_state(cpu, gpu, W, t)
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}: bitstreams differ"
        for p in pg:
            sd.feed(p.data)
        if t == 0 and kind == "desktop":
            assert len(np.unique(qa)) > 1
        assert psnr(sd.Y, bgrx_to_y709(f)) > 28


def _changed_rows(a, b):
    rows = np.nonzero((a != b).any(axis=(1, 2)))[0]
    return [(int(y), int(y) + 1) for y in rows]


def test_gpu_damage_upload_survives_reupload():
    """Damage-driven upload (set_upload_rows): a frame uploaded twice before launch (the
    capture loop retrying with a newer grab) must not leave stale rows in either parity
    buffer. Packets equal the CPU encoder fed the frames that were launched."""
    W, H = 256, 128
    src = SyntheticDesktop(W, H, kind="desktop")
    frames = [np.ascontiguousarray(src.frame(t)) for t in range(8)]
    for t in range(1, 8):   # extra damage in every frame, a different band each time
        frames[t] = frames[t].copy()
        frames[t][(t * 16) % H:(t * 16) % H + 8, :, :3] ^= 0x3C
    cpu, gpu = _pair(W, H, stripe_height=64)
    launched = [0, 1, 3, 4, 6, 7]   # frames 2 and 5 are uploaded, then replaced before launch
    prev = None
    for t in range(8):
        gpu.set_upload_rows(None if prev is None else _changed_rows(frames[prev], frames[t]))
        gpu.upload(frames[t], t)
        prev = t
        if t not in launched:
            continue
        gpu.launch()
        pg = gpu.finish()
        pc = cpu.encode(frames[t], t)
        assert [p.data for p in pg] == [p.data for p in pc], f"frame {t}: HIP packets differ from CPU"
