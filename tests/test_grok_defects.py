"""Grok 9.2.0 defects found by the reviews and what this
repository does instead, checked on the CPU: the oracle's streams against the source image and
cross-decoded by OpenJPEG 2.5.4 (Pillow), an independent decoder.

  R-BUG-5  -T 5,3 -t 128,128 (tile grid offset): Grok's "lossless" stream decodes to 41.3 dB in
           Grok, the oracle and OpenJPEG.  Ours is lossless in all three senses below.
  R-BUG-6  HT -M 64 -t 100,70 (odd-parity tiles, mono16): Grok's stream decodes to 18.1 dB.
  R-BUG-7  -t 24,40: Grok's decoder gives 23.1 dB on a stream (byte-equal to ours) that the
           oracle and OpenJPEG decode losslessly.
  R-BUG-8  rate control whose budget is reached inside a number-of-passes / comma code: Grok's
           simulation misses the failure and writes SOT Psot / TLM / PLT lengths from its own
           count, a few bytes off the tile part.  Reproduced byte for byte (the known answers in
           test_oracle_grok_sizes.py); OpenJPEG rejects such streams, the oracle (and the engine,
           test_gpu_grok_known.py) resynchronise on the next SOT.
  R-BUG-9  ROI with the HT block coder: Grok's RoiShiftHTFilter / RoiScaleHTFilter
           (PostDecompressFilters.h:92-158) test the raw 32-bit decoder sample against 2^shift
           and AND the shifted magnitude with the sign bit, so every region sample decodes to
           zero; its encoder only raises the band bit-plane count (CodeStreamCompress.cpp:538-541).
           Ours is the standard maxshift on the HT indices (test_roi_htj2k_round_trip below); no
           independent decoder pins it (OpenJPEG 2.5.4 refuses RGN with HT), so it is oracle-
           restated and GPU-tested against the oracle (tests/test_gpu_roi.py).
"""
import io

import numpy as np
import pytest

import oracle as O
from conftest import parse_flags
from grok_amd.synth import synth_image

Image = pytest.importorskip("PIL.Image")


def _openjpeg(cs):
    im = Image.open(io.BytesIO(cs))
    im.load()
    a = np.asarray(im).astype(np.int64)
    return a.transpose(2, 0, 1) if a.ndim == 3 else a[None]


def _psnr(a, b, peak):
    mse = ((np.asarray(a, np.float64) - b) ** 2).mean()
    return float("inf") if mse == 0 else 10 * np.log10(peak ** 2 / mse)


@pytest.mark.parametrize("args,bits,flags", [
    ((384, 520, 3, 8, 7), 8, "-T 5,3 -t 128,128"),     # R-BUG-5
    ((300, 260, 1, 16, 21), 16, "-M 64 -t 100,70"),    # R-BUG-6
    ((384, 520, 3, 8, 7), 8, "-t 24,40"),              # R-BUG-7
])
def test_lossless_where_grok_is_not(args, bits, flags):
    img = synth_image(*args).astype(np.int32)
    cs = O.encode(img, bits, **parse_flags(flags))
    dec, _ = O.decode(cs)
    np.testing.assert_array_equal(dec, img)
    np.testing.assert_array_equal(_openjpeg(cs), img)


@pytest.mark.parametrize("flags", ["-t 64,64 -r 40,10", "-t 64,64 -r 40,10 -X -L"])
def test_simulation_counted_lengths_decode(flags):
    # R-BUG-8: at least one tile part's Psot does not lead to the next marker; the oracle's
    # decode resynchronises and gives the layers' quality (about 30.7 dB at 40:1 / 10:1)
    img = synth_image(384, 520, 3, 8, 7).astype(np.int32)
    cs = O.encode(img, 8, **parse_flags(flags))
    pos, bad = cs.find(b"\xff\x90"), 0
    while cs[pos:pos + 2] == b"\xff\x90":
        nxt = pos + int.from_bytes(cs[pos + 6:pos + 10], "big")
        if cs[nxt:nxt + 2] not in (b"\xff\x90", b"\xff\xd9"):
            bad += 1
            nxt = min((q for q in range(nxt - 8, nxt + 9) if cs[q:q + 2] in (b"\xff\x90", b"\xff\xd9")),
                      key=lambda q: abs(q - nxt))
        pos = nxt
    assert bad >= 1
    dec, _ = O.decode(cs)
    assert _psnr(dec, img, 255) > 30.5
    with pytest.raises(Exception):   # OpenJPEG 2.5.4: "broken data stream"
        _openjpeg(cs)


@pytest.mark.parametrize("v,vertical,partial,want", [
    (-3, False, False, -1),   # whole-tile decode: bandH[0] / 2 (WaveletReverse.cpp:583)
    (-3, False, True, -2),    # decode window: Grok's partial-tile path, S(buf, 0) >>= 1 (:1551-1554)
    (-3, True, False, -2),    # down a column both paths shift (:636, :1735)
    (-3, True, True, -2),
    (5, False, False, 2), (5, False, True, 2),
])
def test_single_odd_sample_rule(v, vertical, partial, want):
    # a one-sample line on an odd coordinate holds a high-pass coefficient; Grok halves it
    # differently in its whole-tile and window decodes, and so do the oracle and the engine
    # (gk_dwt_any.hip inv53_line, ctx->dwt_partial)
    assert O.lib().orc_inv53_single(v, 1, int(vertical), int(partial)) == want


@pytest.mark.parametrize("roi,irr", [((0, 4), False), ((1, 6), False), ((2, 3), True)])
def test_roi_htj2k_round_trip(roi, irr):
    # R-BUG-9: the standard maxshift on HT indices; 5/3 lossless, 9/7 at its usual distortion, and
    # the same image without ROI decodes alike (the shift only lifts the region above background)
    img = synth_image(120, 136, 3, 8, 90 + roi[1]).astype(np.int32)
    cs = O.encode(img, 8, numres=4, irreversible=irr, roi=roi, cblk_sty=0x40)
    assert b"\xff\x5e" in cs
    dec, _ = O.decode(cs)
    plain, _ = O.decode(O.encode(img, 8, numres=4, irreversible=irr, cblk_sty=0x40))
    if not irr:
        np.testing.assert_array_equal(dec, img)
    np.testing.assert_array_equal(dec, plain)
