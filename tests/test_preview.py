"""Preview path: aspect-fit size, the GUI's gamma table,
the oracle's preview tail, and (gpu) libh2s vs the oracle.

PARITY UNPINNED for the resize and the yuv420p->rgb24 step: no ffmpeg or
swscale exists in this image. Pinned: the scale box arithmetic (ffmpeg's
force_original_aspect_ratio=decrease formula, cases below) and the display
gamma, which is checked against PIL itself applying the reference's
adjust_gamma table (src/preview.py:108-117)."""
import math

import numpy as np
import pytest

import oracle
import hdr2sdr
from hdr2sdr import preview as PV
from hdr2sdr.synth import synth_frames


@pytest.mark.parametrize('iw,ih,bw,bh,want', [
    (3840, 2160, 3840, 2160, (3840, 2160)),     # 4K source: no-op scale
    (7680, 4320, 3840, 2160, (3840, 2160)),     # 8K: downscale
    (1920, 1080, 3840, 2160, (3840, 2160)),     # 1080p: upscaled to the box
    (3840, 1608, 3840, 2160, (3840, 1608)),     # scope: width-limited
    (4096, 2160, 3840, 2160, (3840, 2025)),     # DCI 4K: av_rescale(3840, 2160, 4096) = 2025
    (1440, 1080, 960, 540, (720, 540)),         # 4:3 in a 16:9 box
    (3840, 2160, 'iw', 'ih', (3840, 2160)),
])
def test_fit_size(iw, ih, bw, bh, want):
    bw = iw if bw == 'iw' else bw
    bh = ih if bh == 'ih' else bh
    assert PV.fit_size(iw, ih, bw, bh) == want


def test_fit_size_rejects_nonpositive():
    with pytest.raises(ValueError):
        PV.fit_size(0, 1080)


@pytest.mark.parametrize('gamma', [1.0, 2.2, 0.5, 1.3])
def test_display_gamma_matches_pil_adjust_gamma(gamma):
    """The fused table equals what PIL's point() does with the reference's
    adjust_gamma list, checked on every 8-bit value."""
    from PIL import Image
    img = Image.fromarray(np.arange(256, dtype=np.uint8).reshape(16, 16).repeat(3).reshape(16, 16, 3), 'RGB')
    if abs(gamma - 1.0) < 1e-6:
        ref = img
    else:
        lut = [pow(i / 255.0, 1.0 / gamma) * 255 for i in range(256)] * 3
        ref = img.point([int(round(v)) for v in lut])
    want = np.asarray(ref)[..., 0].reshape(-1)
    assert np.array_equal(PV.adjust_gamma_lut(gamma), want)
    # and the oracle's preview tail applies the same table: a mid-grey frame
    # (Y=126, neutral chroma) -> RGB 128 before the table
    W, H = 4, 4
    yuv = np.concatenate([np.full(W * H, 126, np.uint8), np.full(W * H // 2, 128, np.uint8)])
    out = np.zeros((H, W, 3), np.uint8)
    assert oracle.lib().oracle_preview_tail(yuv.ctypes.data, W, H, W, H, gamma, out.ctypes.data) == 0
    assert np.all(out == want[128])


def test_oracle_preview_tail_resize_preserves_flat_fields():
    W, H = 64, 32
    yuv = np.concatenate([np.full(W * H, 100, np.uint8), np.full(W * H // 4, 90, np.uint8),
                          np.full(W * H // 4, 170, np.uint8)])
    for ow, oh in ((32, 16), (128, 64), (50, 25)):
        out = np.zeros((oh, ow, 3), np.uint8)
        assert oracle.lib().oracle_preview_tail(yuv.ctypes.data, W, H, ow, oh, 1.0, out.ctypes.data) == 0
        assert np.all(out == out[0, 0])     # a flat field stays flat through any resize


_LAT = {}


def _lat():
    if 65 not in _LAT:
        _LAT[65] = hdr2sdr.generate_lattice(65)
    return _LAT[65]


PREVIEW_CASES = [
    (256, 128, (256, 128), 'reinhard', True),    # source-size preview (the 4K->4K case)
    (512, 256, (256, 128), 'mobius', True),      # downscale (the 8K->4K case)
    (128, 64, (256, 128), 'reinhard', True),     # upscale (1080p->4K)
    (384, 256, (256, 144), 'hable', False),      # aspect fit + legacy no-LUT chain
]


def _gpu_chain_yuv8(params, src, W, H):
    """The GPU's own 8-bit chain output for frame 0 (the preview's input)."""
    tm = hdr2sdr.Tonemapper(0, params, _lat() if params.lut_enabled else None)
    out = hdr2sdr.FrameBatch.empty_numpy(1, W, H, 8)
    tm.process(hdr2sdr.FrameBatch(np.ascontiguousarray(src.buf[:1]), W, H, src.bits), out)
    tm.close()
    return np.ascontiguousarray(out.buf[0])


@pytest.mark.gpu
@pytest.mark.parametrize('W,H,box,tm,lut', PREVIEW_CASES)
def test_gpu_preview_tail_matches_oracle_tail(W, H, box, tm, lut):
    """Resize + yuv420p->rgb24 alone: the oracle tail applied to the GPU's
    own chain output.  Same size: identical.  Resized: fp32 vs fp64 filter
    weights may move a resized Y/U/V sample by 1, i.e. R/G/B by up to
    ceil(1.164 + 2.112) = 4, on a small fraction of pixels."""
    src = synth_frames('smooth', 1, W, H, 10, device='cpu', seed=3).to_numpy()
    with PV.Previewer(0, tonemapper=tm, lut_enabled=lut, lattice=_lat()) as pv:
        got = pv.convert(src, box[0], box[1])
        ow, oh = PV.fit_size(W, H, *box)
        yuv8 = _gpu_chain_yuv8(pv.params, src, W, H)
    want = np.zeros((oh, ow, 3), np.uint8)
    assert oracle.lib().oracle_preview_tail(yuv8.ctypes.data, W, H, ow, oh, 1.0, want.ctypes.data) == 0
    d = np.abs(got.astype(int) - want.astype(int))
    if (ow, oh) == (W, H):
        assert d.max() <= 1 and (d > 0).mean() < 1e-3
    else:
        assert d.max() <= 4 and (d > 0).mean() < 2e-2


@pytest.mark.gpu
@pytest.mark.parametrize('gamma', [2.2, 0.5, 1.3])
def test_gpu_preview_display_gamma_is_the_pil_table(gamma):
    src = synth_frames('smooth', 1, 256, 128, 10, device='cpu', seed=8).to_numpy()
    with PV.Previewer(0, tonemapper='hable', lattice=_lat()) as pv:
        base = pv.convert(src, 'iw', 'ih', gamma=1.0)
        got = pv.convert(src, 'iw', 'ih', gamma=gamma)
    assert np.array_equal(got, PV.adjust_gamma_lut(gamma)[base])


@pytest.mark.gpu
@pytest.mark.parametrize('W,H,box,tm,lut', PREVIEW_CASES)
def test_gpu_preview_end_to_end_vs_oracle(W, H, box, tm, lut):
    """Chain + tail vs the oracle's chain + tail: the chain's +-1 step in
    Y/Cb/Cr moves R/G/B by at most ceil(1.164 + 2.112) = 4."""
    src = synth_frames('smooth', 1, W, H, 10, device='cpu', seed=3).to_numpy()
    with PV.Previewer(0, tonemapper=tm, lut_enabled=lut, lattice=_lat()) as pv:
        got = pv.convert(src, box[0], box[1])
        ow, oh = PV.fit_size(W, H, *box)
        want = oracle.preview_rgb24(oracle.params_from(pv.params.to_c()), _lat() if lut else None, src.buf, W, H,
                                    ow, oh, 1.0)
    d = np.abs(got.astype(int) - want.astype(int))
    assert d.max() <= 4 and (d > 1).mean() < 1e-2


@pytest.mark.gpu
def test_gpu_preview_rejects_non_8bit_context():
    src = synth_frames('smooth', 1, 128, 64, 10, device='cpu', seed=3).to_numpy()
    tm = hdr2sdr.Tonemapper(0, hdr2sdr.TonemapParams(tonemapper='hable', bits_out=10), _lat())
    out = np.empty((64, 128, 3), np.uint8)
    import ctypes
    from hdr2sdr import _abi
    d = src.descriptor()
    rc = _abi.lib().h2s_preview_rgb24(tm._ctx, ctypes.byref(d), out.ctypes.data, 3 * 128, 128, 64, 1.0,
                                      _abi.LOC_HOST, None)
    assert rc == _abi.H2S_E_INVALID_ARG
    tm.close()


@pytest.mark.gpu
@pytest.mark.parametrize('kind,seed', [('smooth', 21), ('ramp', 5)])
def test_gpu_lut_chain_tracks_legacy_gamut_chain(kind, seed):
    """The reference's colour-correctness safety net,
    TestLutReproducesLegacyGamutMath (test/smoke_test.py:264-343), on the
    product path: one 960x540 HDR10 frame through libh2s as the reference
    renders it to PNG, once with FFMPEG_CONVERT_FILTER (reinhard, gamma 1,
    65^3 tetrahedral LUT: k_tile) and once with FFMPEG_FILTER_LEGACY_NO_LUT
    (closed-form BT.2020->709 + clip), sampled on the same 21x21 grid
    (w // 20 steps); max per-channel difference <= 12/255 (_TOLERANCE,
    :300).  The reference measured a worst case of 10/255 on real content."""
    W, H = 960, 540
    src = synth_frames(kind, 1, W, H, 10, device='cpu', seed=seed).to_numpy()
    imgs = []
    for lut in (False, True):
        with PV.Previewer(0, tonemapper='reinhard', lut_enabled=lut, lattice=_lat()) as pv:
            imgs.append(pv.convert(src, 'iw', 'ih').astype(int))
    legacy, with_lut = imgs
    xs = np.arange(0, W, max(1, W // 20))
    ys = np.arange(0, H, max(1, H // 20))
    d = np.abs(legacy[ys][:, xs] - with_lut[ys][:, xs])
    assert d.max() <= 12, f'LUT chain differs from the legacy chain by up to {d.max()}/255'
    assert np.abs(legacy - with_lut).mean() < 3.0        # and close on average, not only on the grid


@pytest.mark.gpu
@pytest.mark.parametrize('tm,use_gpu', [('reinhard', False), ('bt.2390', False), ('hable', True)])
def test_gpu_preview_batch_mixed_sizes_vs_oracle(tm, use_gpu):
    """The batched preview (extract_frames_with_conversion_batch /
    extract_frames_with_gpu_conversion_batch, src/utils.py:668-716, :803-824):
    N = 4 frames of two sizes in one convert_batch call (one libh2s call per
    size), each against the oracle's chain + preview tail for that frame
    alone, and bit-identical to converting it on its own.  The libplacebo
    preview (bt.2390; hable with GPU tone mapping on) detects each frame's
    peak from a fresh state, as the reference's per-frame ffmpeg runs do."""
    sizes = [(256, 128), (384, 256), (256, 128), (384, 256)]
    frames = [synth_frames('smooth', 1, w, h, 10, device='cpu', seed=60 + i).to_numpy()
              for i, (w, h) in enumerate(sizes)]
    box = (192, 108)
    with PV.Previewer(0, tonemapper=tm, use_gpu=use_gpu, lattice=_lat()) as pv:
        assert pv.params.peak_detect == (tm == 'bt.2390' or use_gpu)
        batch = pv.convert_batch(frames, *box)
        singles = [pv.convert(f, *box) for f in frames]
        batch13 = pv.convert_batch(frames, *box, gamma=1.3)
        op = oracle.params_from(pv.params.to_c())
    g13 = PV.adjust_gamma_lut(1.3)
    for f, (w, h), got, one, got13 in zip(frames, sizes, batch, singles, batch13):
        ow, oh = pv.out_size(w, h, *box)
        # the libplacebo preview outputs exactly the box (vf_libplacebo w/h,
        # no aspect option: src/utils.py:787); the CPU chain fits the aspect
        assert (ow, oh) == (box if pv.params.resolved_pipeline() == 'libplacebo' else PV.fit_size(w, h, *box))
        assert got.shape == (oh, ow, 3)
        assert np.array_equal(got, one)
        assert np.array_equal(got13, g13[got])          # the display gamma, fused
        want = oracle.preview_rgb24(op, _lat(), f.buf, w, h, ow, oh, 1.0)
        d = np.abs(got.astype(int) - want.astype(int))
        assert d.max() <= 4 and (d > 1).mean() < 1e-2


@pytest.mark.gpu
def test_gpu_preview_batch_one_size_is_one_frame_batch():
    """Frames of one FrameBatch go through as one batch: equal to their
    single-frame previews."""
    src = synth_frames('smooth', 3, 256, 128, 10, device='cpu', seed=9).to_numpy()
    with PV.Previewer(0, tonemapper='hable', lattice=_lat()) as pv:
        batch = pv.convert_batch(src, 'iw', 'ih')
        singles = [pv.convert(src.slice(i, i + 1), 'iw', 'ih') for i in range(3)]
    assert len(batch) == 3 and all(np.array_equal(a, b) for a, b in zip(batch, singles))
