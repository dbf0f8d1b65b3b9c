"""CPU tests of the host side: librdmi loads and exports every entry point include/rdmi.h declares
(no compute calls without a GPU), weight packing layouts, snippet scheduling, DDIM coefficients,
sharding partition logic."""
import os
import re

import numpy as np
import pytest
import torch

from oracle import rd_oracle as O

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_library_exports_every_header_symbol():
    from rollingdepth_amd import _native

    hdr = open(os.path.join(ROOT, "include", "rdmi.h")).read()
    declared = set(re.findall(r"\b(rdmi_[a-z0-9_]+)\s*\(", hdr))
    assert declared, "no declarations parsed"
    for name in declared:
        assert hasattr(_native.lib, name), f"librdmi.so does not export {name}"
    assert declared == set(_native.EXPORTED), declared ^ set(_native.EXPORTED)
    assert _native.lib.rdmi_version() >= 1


def test_error_reporting_without_gpu():
    """Argument validation runs before any launch, so bad calls fail loudly on the host."""
    import ctypes as C
    from rollingdepth_amd import _native

    g = _native.GemmArgs()
    rc = _native.lib.rdmi_gemm(C.byref(g), None)
    assert rc == 1001
    assert b"null" in _native.lib.rdmi_last_error()
    with pytest.raises(_native.RdmiError):
        _native.check(rc, "rdmi_gemm")


def test_pack_conv_layout():
    from rollingdepth_amd import kernels as K

    w = torch.randn(5, 3, 3, 3)
    p = K.pack_conv(w, "cpu", 8)
    assert p.shape == (5, 96)
    t = p[:, :72].float().view(5, 3, 3, 8)
    assert torch.allclose(t[..., :3], w.permute(0, 2, 3, 1).half().float())
    assert t[..., 3:].abs().max() == 0 and p[:, 72:].abs().max() == 0


def test_pack_conv_channel_block_major():
    """Cin % 64 == 0, 3x3: K order [Cin/64][kh][kw][64] (rdmi.h conv weight layout)."""
    from rollingdepth_amd import kernels as K

    w = torch.randn(4, 128, 3, 3)
    p = K.pack_conv(w, "cpu")
    assert p.shape == (4, 1152)
    t = p.float().view(4, 2, 3, 3, 64)
    for cb in range(2):
        for dy in range(3):
            for dx in range(3):
                assert torch.equal(t[:, cb, dy, dx], w[:, cb * 64:(cb + 1) * 64, dy, dx].half().float())
    # Cin % 64 != 0 keeps the tap-major order
    w3 = torch.randn(2, 32, 3, 3)
    assert torch.equal(K.pack_conv(w3, "cpu").float().view(2, 3, 3, 32), w3.permute(0, 2, 3, 1).half().float())
    # 1x1 kernels keep the plain [Cout][Cin] order
    w1 = torch.randn(3, 64, 1, 1)
    assert torch.equal(K.pack_conv(w1, "cpu").float(), w1[:, :, 0, 0].half().float())


def test_split_bf16_layout(monkeypatch):
    """RDMI_F32_X3 weights (rdmi.h): per 32-deep K-tile, 32 bf16 hi then 32 bf16 lo; hi + lo is the
    f32 weight to ≈2^-17 relative; zero K padding stays zero in both parts."""
    from rollingdepth_amd import kernels as K

    w = torch.randn(6, 70) * torch.logspace(-3, 3, 70)
    monkeypatch.setenv("RDMI_F32_X3", "0")
    f = K.pack_linear(w, "cpu", torch.float32)
    monkeypatch.setenv("RDMI_F32_X3", "1")
    p = K.pack_linear(w, "cpu", torch.float32)
    assert f.shape == (6, 96) and p.shape == (6, 192) and p.dtype == torch.bfloat16
    t = p.view(6, 3, 2, 32).float()
    hi, lo = t[:, :, 0].reshape(6, 96), t[:, :, 1].reshape(6, 96)
    assert torch.equal(hi, f.to(torch.bfloat16).float())
    assert ((hi + lo - f).abs() <= f.abs() * 2.0 ** -16).all()
    assert hi[:, 70:].abs().max() == 0 and lo[:, 70:].abs().max() == 0
    c = K.pack_conv(torch.randn(4, 40, 3, 3), "cpu", 40, torch.float32)
    assert c.dtype == torch.bfloat16 and c.shape == (4, 2 * 384)


def test_split_weight_engine_from_row_length():
    """The x3 / x6 engine is chosen from the bf16 weight's row length (2·Kp / 4·Kp), so a copy that
    lost the `_rdmi_parts` tag still runs the right engine; a row length matching neither layout, or a
    tag contradicting it, raises instead of running an engine on the wrong layout."""
    from rollingdepth_amd import kernels as K

    w = torch.randn(6, 70)
    x3 = K.split_bf16(torch.nn.functional.pad(w, (0, 26)))
    x6 = K.split3_bf16(torch.nn.functional.pad(w, (0, 26)))
    assert K.split_parts(x3, 70) == 2
    assert K.split_parts(x6, 70) == 3
    assert K.split_parts(x6.clone(), 70) == 3  # the clone dropped the tag
    with pytest.raises(ValueError):
        K.split_parts(x3[:, :160], 70)
    bad = x3.clone()
    bad._rdmi_parts = 3
    with pytest.raises(ValueError):
        K.split_parts(bad, 70)


def test_pack_conv_up2_phase_identity():
    """pack_conv_up2: conv3×3(nearest×2(x)) == the four 2×2 phase convs on the source grid with
    merged weights hi + lo (rdmi.h rdmi_conv_args.w_up2) — the identity the GPU's phase-decomposed
    upsample relies on, checked in f64 against the 9-tap conv of the f16-rounded weights (what the
    9-tap kernel multiplies by), and the [phase][Cout][Cin/64][7][64] layout."""
    from rollingdepth_amd import kernels as K

    torch.manual_seed(0)
    B, Cin, Cout, H, W = 2, 128, 8, 5, 7
    x = torch.randn(B, Cin, H, W, dtype=torch.float64)
    w = torch.randn(Cout, Cin, 3, 3) * 0.05
    wu = K.pack_conv_up2(w, "cpu")
    assert wu.shape == (4, Cout, 7 * Cin) and wu.dtype == torch.float16
    t7 = wu.double().view(4, Cout, Cin // 64, 7, 64)
    wph = torch.zeros(4, Cout, Cin // 64, 4, 64, dtype=torch.float64)
    for ph in range(4):
        wph[ph] = t7[ph, :, :, :4]
        lo_taps = [t for t in range(4) if t != ph]  # lo parts in tap order, the phase's own tap has none
        for s_, t in enumerate(lo_taps):
            wph[ph, :, :, t] += t7[ph, :, :, 4 + s_]
    wph = wph.view(4, Cout, Cin // 64, 2, 2, 64).permute(0, 1, 2, 5, 3, 4).reshape(4, Cout, Cin, 2, 2)
    w16 = w.half().double()
    ref = torch.nn.functional.conv2d(torch.nn.functional.interpolate(x, scale_factor=2.0, mode="nearest"),
                                     w16, padding=1)
    xp = torch.nn.functional.pad(x, (1, 1, 1, 1))
    got = torch.empty_like(ref)
    for a in range(2):
        for c in range(2):
            got[:, :, a::2, c::2] = torch.nn.functional.conv2d(xp[:, :, a:a + H + 1, c:c + W + 1], wph[2 * a + c])
    # hi + lo carries each merged weight to within lo's own f16 rounding (≤ 2^-22 of it here)
    assert (got - ref).abs().max().item() < 1e-6 * ref.abs().max().item()
    # the phase's single-weight tap is the f16 weight itself; a 4-weight tap is hi + lo of the exact sum
    assert torch.equal(t7[0, :, :, 0], w16[:, :, 0, 0].reshape(Cout, 2, 64))
    s4 = w16[:, :, 1:, 1:].sum((2, 3))
    assert torch.equal(t7[0, :, :, 3], s4.half().double().reshape(Cout, 2, 64))
    assert torch.equal(t7[0, :, :, 6], (s4 - s4.half().double()).half().double().reshape(Cout, 2, 64))
    assert torch.equal(t7[3, :, :, 3], w16[:, :, 2, 2].reshape(Cout, 2, 64))
    assert K.pack_conv_up2(torch.randn(4, 32, 3, 3), "cpu") is None  # Cin_pad % 64 != 0


def test_geglu_permutation_roundtrip():
    from rollingdepth_amd import kernels as K

    w = torch.arange(256 * 2).float().view(256, 2)
    b = torch.arange(256).float()
    wp, bp = K.geglu_permute(w, b)
    # slab s: value rows 32s..32s+31 then gate rows 128+32s..
    assert torch.equal(bp[:32], b[:32]) and torch.equal(bp[32:64], b[128:160])
    assert sorted(bp.tolist()) == b.tolist()


def test_snippet_scheduling_matches_golden():
    import json
    from rollingdepth_amd.pipeline import RollingDepthPipeline as P

    idx = json.load(open(os.path.join(ROOT, "tests", "golden", "snippet_indices.json")))
    for n, w, d, capped in idx["cap"]:
        assert P.cap_max_dilation(n, w, d) == capped
    for n, spec, expect in idx["snippets"]:
        if isinstance(spec, list):
            ds, de, i_step, T = spec
            assert P.get_snippet_indice(i_step, list(range(T)), n, 3, ds, de, 1) == expect
        else:
            assert P.get_snippet_indice(0, [999], n, 3, spec, spec, 1) == expect


def test_ddim_coefficients_vs_oracle():
    from rollingdepth_amd.config import RD_SCHEDULER
    from rollingdepth_amd.scheduler import DDIMScheduler

    s = DDIMScheduler.from_config(RD_SCHEDULER)
    o = O.DDIM(RD_SCHEDULER)
    x, e = torch.randn(1000), torch.randn(1000)
    for n in (1, 10):
        s.set_timesteps(n)
        ts = o.set_timesteps(n)
        assert s.timesteps.tolist() == ts
        for t in ts:
            ca, cb = s.step_coefficients(t)
            torch.testing.assert_close(ca * x + cb * e, o.step(e, t, x), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("counts,world", [([98, 50], 1), ([98, 50], 2), ([98, 50], 8), ([498, 480, 450], 8),
                                          ([7, 5], 4), ([3], 8)])
def test_shard_partition_covers_every_snippet_once(counts, world):
    from rollingdepth_amd.shard import chunk_bounds, flat_snippets, rank_subsets

    seen = []
    for r in range(world):
        sub = rank_subsets(counts, world, r)
        for d, ks in enumerate(sub):
            assert ks == sorted(ks) and (not ks or ks == list(range(ks[0], ks[-1] + 1)))
            seen += [(d, k) for k in ks]
    assert seen == flat_snippets(counts)
    sizes = [hi - lo for lo, hi in chunk_bounds(sum(counts), world)]
    assert max(sizes) - min(s for s in sizes if s) <= max(1, max(sizes))


def test_empty_text_embedding_vs_transformers_and_reference(tmp_path):
    """encode_empty_text restated (rollingdepth_amd/text_encoder.py): tokenizer("") → [BOS, EOS] and the
    CLIP text transformer on those two tokens — against transformers' CLIPTokenizer + CLIPTextModel
    (the reference's own classes, rollingdepth_pipeline.py:178-191) on the same synthesised weights,
    and against the context the reference pipeline computed for the tiny_clip_pipeline fixture."""
    import json

    from safetensors.torch import load_file

    from rollingdepth_amd import text_encoder as TE
    from tests.ckpt_util import write_text_encoder

    meta = json.load(open(os.path.join(ROOT, "tests", "golden", "tiny_clip_pipeline.json")))
    ref_ctx = load_file(os.path.join(ROOT, "tests", "golden", "tiny_clip_pipeline.safetensors"))["context"]
    write_text_encoder(str(tmp_path), meta["text_encoder"], meta["tokenizer_vocab"], meta["text_encoder_seed"])
    got = TE.empty_text_embedding(str(tmp_path))
    assert got.shape == ref_ctx.shape == (1, 2, 96)
    assert (got - ref_ctx).abs().max().item() < 1e-5
    transformers = pytest.importorskip("transformers")
    tk = transformers.CLIPTokenizer.from_pretrained(str(tmp_path / "tokenizer"))
    ids = tk("", padding="do_not_pad", max_length=tk.model_max_length, truncation=True, return_tensors="pt").input_ids
    assert ids.tolist() == [list(TE.special_token_ids(str(tmp_path / "tokenizer")))]
    # SD2-sized text tower (1024 wide, 23 layers, OpenCLIP ViT-H's gelu) on synthesised weights
    cfg = dict(meta["text_encoder"], hidden_size=1024, intermediate_size=4096, num_hidden_layers=23,
               num_attention_heads=16)
    big = tmp_path / "sd2"
    write_text_encoder(str(big), cfg, meta["tokenizer_vocab"], 3)
    m = transformers.CLIPTextModel(transformers.CLIPTextConfig(**cfg)).eval()
    sd = load_file(str(big / "text_encoder" / "model.safetensors"))
    own = set(m.state_dict())
    m.load_state_dict({(k if k in own else k[len("text_model."):]): v for k, v in sd.items()}, strict=True)
    with torch.no_grad():
        want = m(ids)[0]
    got = TE.empty_text_embedding(str(big))
    assert (got - want).abs().max().item() < 2e-5 * max(1.0, want.abs().max().item())


def test_video_target_size_and_missing_pyav():
    """video_io.py:58-65 target size (Python float arithmetic) and the loud PyAV boundary."""
    from rollingdepth_amd import video_io as V

    for (h, w, r) in [(1080, 1920, 768), (1080, 1920, 1024), (720, 1280, 768), (331, 197, 120), (100, 100, 768)]:
        f = min(r / w, r / h)
        assert V._target_size(h, w, r) == (int(h * f), int(w * f))
    assert V._target_size(1080, 1920, 768) == (432, 768)
    try:
        import av  # noqa: F401
    except ImportError:
        with pytest.raises(ImportError, match="PyAV"):
            V.load_video_frames("/nonexistent.mp4")
        with pytest.raises(ImportError, match="PyAV"):
            V.write_video_from_numpy(np.zeros((1, 4, 4, 3), np.uint8), "/tmp/x.mp4")
    with pytest.raises(ValueError):
        V.frames_from_rgb24(np.zeros((1, 4, 4, 4), np.uint8))


def test_aligner_workspace_sizes_history_slots():
    """rdmi_aligner_workspace (host-only, no GPU): the fused aligner loop keeps per-iteration loss
    partials (2·ntot·PS doubles), chunk min/max (2·N·PS floats) and pre-update parameters (2·ntot)
    for one block of at most 128 iterations when a history is requested (aligner.hip HBLK: the
    workspace does not grow with the iteration count), and nothing per iteration without one — but
    the Adam bias-correction table, 2 doubles per iteration (adam_bc_k)."""
    import ctypes as C

    from rollingdepth_amd import _native

    a = _native.AlignerArgs()
    a.n_dil, a.seq_len, a.P = 2, 100, 5929
    a.w[0], a.w[1] = 3, 3
    a.n[0], a.n[1] = 98, 48
    ntot, PS = 146, 8
    a.iters = 2000
    a.history = None
    base = _native.lib.rdmi_aligner_workspace(C.byref(a))
    assert base >= 8 * ntot * PS + 8 * 100 * PS + 2 * 100 * 5929 + 4 * ntot + ntot + 4 * 2001
    a.history = 1  # any non-null pointer: the size depends only on its presence
    with_hist = _native.lib.rdmi_aligner_workspace(C.byref(a))
    per_it = 4 * ntot * PS + 2 * 100 * PS + 2 * ntot
    assert 128 * per_it <= with_hist - base <= 128 * per_it + 64
    a.iters = 128
    assert _native.lib.rdmi_aligner_workspace(C.byref(a)) == with_hist - 4 * (2000 - 128)
    a.iters = 10
    assert _native.lib.rdmi_aligner_workspace(C.byref(a)) < with_hist


def test_colorize_rejects_float64():
    """The device colouriser evaluates the reference's index arithmetic in f16 / f32; float64 depth
    (which the reference normalises in float64) is refused instead of silently rounded (no GPU call:
    the dtype check precedes any device work)."""
    import numpy as np

    from rollingdepth_amd import colorize as Cz

    with pytest.raises(TypeError, match="float64"):
        Cz.colorize_depth_multi_thread(np.zeros((1, 1, 4, 4)), device="cpu")
    with pytest.raises(TypeError, match="float64"):
        Cz.colorize_depth(np.zeros((1, 4, 4)), 0.0, 1.0, device="cpu")


class _FakeAV:
    """Stand-in for PyAV (absent from the image) recording what write_video_from_numpy asks of it:
    the codec fallback, stream settings, every encoded frame and the flush."""

    def __init__(self, known=("mpeg4", "mjpeg")):
        import types

        self.known, self.log, self.frames = set(known), [], []

        class UnknownCodecError(Exception):
            pass

        self.codec = types.SimpleNamespace(codec=types.SimpleNamespace(UnknownCodecError=UnknownCodecError))
        av = self

        class Stream:
            def encode(self, frame):
                av.log.append(("encode", frame is None))
                if frame is not None:
                    av.frames.append(frame.arr.copy())
                return [("packet", len(av.log))]

        class Container:
            def add_stream(self, codec, rate):
                av.log.append(("add_stream", codec, rate))
                if codec not in av.known:
                    raise UnknownCodecError(codec)
                av.stream = Stream()
                return av.stream

            def mux(self, packet):
                av.log.append(("mux",))

            def close(self):
                av.log.append(("close",))

        class VideoFrame:
            @staticmethod
            def from_ndarray(arr, format):
                assert format == "rgb24"
                return type("F", (), {"arr": arr})()

        self.open = lambda path, mode="r": (self.log.append(("open", path, mode)), Container())[1]
        self.VideoFrame = VideoFrame


def test_write_video_from_numpy_against_a_pyav_stand_in(monkeypatch):
    """video_io.py:140-208's encoder loop through a recording stand-in for PyAV: codec fallback past
    the x264 codecs, yuv420p, no x264 options on mpeg4, one rgb24 frame per input in order, flush."""
    import sys

    import numpy as np

    from rollingdepth_amd import video_io as V

    fake = _FakeAV()
    monkeypatch.setitem(sys.modules, "av", fake)
    frames = (np.arange(3 * 4 * 6 * 3) % 251).astype(np.uint8).reshape(3, 4, 6, 3)
    V.write_video_from_numpy(frames, "/tmp/out.mp4", fps=12)
    tried = [e[1] for e in fake.log if e[0] == "add_stream"]
    assert tried == ["libx264", "h264", "mpeg4"]
    st = fake.stream
    assert (st.width, st.height, st.pix_fmt) == (6, 4, "yuv420p") and not hasattr(st, "options")
    assert len(fake.frames) == 3 and all(np.array_equal(a, b) for a, b in zip(fake.frames, frames))
    enc = [e for e in fake.log if e[0] == "encode"]
    assert enc[-1] == ("encode", True) and len(enc) == 4
    assert fake.log[-1] == ("close",)
    fake2 = _FakeAV(known=("libx264",))
    monkeypatch.setitem(sys.modules, "av", fake2)
    V.write_video_from_numpy(frames, "/tmp/out.mp4", crf=18, preset="fast")
    assert fake2.stream.options == {"crf": "18", "preset": "fast"}
    monkeypatch.setitem(sys.modules, "av", _FakeAV(known=()))
    with pytest.raises(ValueError, match="No working codec"):
        V.write_video_from_numpy(frames, "/tmp/out.mp4")
