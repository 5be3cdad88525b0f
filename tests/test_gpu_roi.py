"""Region of interest, maxshift (RGN marker, grk_compress -ROI c=<comp>,U=<shift>): the
whole component is the region.  Decode follows Grok's RoiShiftFilter / RoiScaleFilter
(PostDecompressFilters.h:7-72: a decoded sample at or above 2^shift is shifted down);
encode is the standard-correct maxshift (the integer part of the component's indices scaled
by 2^shift, band bit-plane count raised by the shift), where Grok's encoder only raises the
bit-plane count (CodeStreamCompress.cpp:538-541) and so distorts its own ROI streams.
Bar: HIP encode byte-identical to the oracle, decode sample-identical, 5/3 lossless."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("roi", [(0, 5), (1, 3), (2, 10)])
@pytest.mark.parametrize("irr", [False, True])
def test_roi_vs_oracle(eng, roi, irr):
    import grok_amd as G
    rng = np.random.default_rng(roi[1])
    yy, xx = np.mgrid[0:120, 0:140]
    img = np.clip((np.sin(xx / 9.0) + 1)[None] * 100 + rng.integers(0, 40, size=(3, 120, 140)), 0, 255).astype(np.int32)
    cs = eng.encode(img, 8, params=G.default_params(numresolution=4, irreversible=irr, roi=roi))
    ref = O.encode(img, 8, numres=4, irreversible=irr, roi=roi)
    assert cs == ref
    assert b"\xff\x5e" in cs
    dec = eng.decode(cs)
    np.testing.assert_array_equal(dec, O.decode(cs)[0])
    if not irr:
        np.testing.assert_array_equal(dec, img)
    else:
        assert np.abs(dec.astype(np.int64) - img).max() <= 6


def test_roi_mode_switch_path(eng):
    """the mode-switch T1 kernels apply the same scaling and filter"""
    import grok_amd as G
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=(1, 64, 96)).astype(np.int32)
    cs = eng.encode(img, 8, params=G.default_params(numresolution=3, cblk_sty=5, roi=(0, 4)))
    assert cs == O.encode(img, 8, numres=3, cblk_sty=5, roi=(0, 4))
    np.testing.assert_array_equal(eng.decode(cs), img)


def test_roi_component_past_last_is_ignored(eng):
    """grk_cparameters::roi_compno past the last component matches no component
    (CodeStreamCompress.cpp:538-541 compares it with each index), so no RGN is written."""
    import grok_amd as G
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, size=(3, 48, 40)).astype(np.int32)
    plain = eng.encode(img, 8, params=G.default_params(numresolution=3))
    for c in (3, 1 << 30):
        cs = eng.encode(img, 8, params=G.default_params(numresolution=3, roi=(c, 7)))
        assert cs == plain and b"\xff\x5e" not in cs


def _split_marker(cs, code):
    """(offset, length incl. marker) of the first main-header marker `code`"""
    i = 2
    while True:
        m, L = int.from_bytes(cs[i:i + 2], "big"), int.from_bytes(cs[i + 2:i + 4], "big")
        if m == code:
            return i, 2 + L
        assert m != 0xff90
        i += 2 + L


def test_rgn_in_tile_part_header(eng):
    """RGN moved from the main header into the tile-part header: the tile's own ROI shift
    (read_rgn on the tile's tcp, CodeStreamDecompress.cpp:1476-1520): the stream decodes as before,
    as the oracle decodes it."""
    import grok_amd as G
    rng = np.random.default_rng(6)
    img = rng.integers(0, 256, size=(1, 40, 48)).astype(np.int32)
    cs = eng.encode(img, 8, params=G.default_params(numresolution=3, roi=(0, 4)))
    o, n = _split_marker(cs, 0xff5e)
    rgn = cs[o:o + n]
    body = cs[:o] + cs[o + n:]
    sot = body.index(b"\xff\x90")
    psot = int.from_bytes(body[sot + 6:sot + 10], "big")
    sot_new = body[sot:sot + 6] + ((psot + n) if psot else 0).to_bytes(4, "big") + body[sot + 10:sot + 12]
    spliced = body[:sot] + sot_new + rgn + body[sot + 12:]
    np.testing.assert_array_equal(eng.decode(spliced), O.decode(spliced)[0])
    np.testing.assert_array_equal(eng.decode(spliced), img)
    np.testing.assert_array_equal(eng.decode(cs), img)


def test_band_bitplanes_over_30_refused(eng):
    """A Part-1 stream whose band bit-plane count (QCD exponent + guard bits - 1, plus the ROI
    shift) exceeds 30 cannot be held as (2M+1) << q in an int32: refused, not decoded."""
    import grok_amd as G
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, size=(1, 40, 48)).astype(np.int32)
    cs = eng.encode(img, 8, params=G.default_params(numresolution=3, roi=(0, 10)))
    np.testing.assert_array_equal(eng.decode(cs), img)
    o, n = _split_marker(cs, 0xff5e)
    bad = cs[:o + n - 1] + bytes([29]) + cs[o + n:]   # shift 29: HH numbps 29 + 11 > 30
    with pytest.raises(RuntimeError, match="30 band bit-planes"):
        eng.decode(bad)
    np.testing.assert_array_equal(eng.decode(cs), img)


@pytest.mark.parametrize("roi", [(0, 4), (1, 7), (2, 2)])
@pytest.mark.parametrize("irr", [False, True])
def test_roi_htj2k_vs_oracle(eng, roi, irr):
    """ROI with the HT block coder (standard-correct maxshift on the indices, CAP's MAGBp raised by
    the shift; Grok's RoiShiftHTFilter keeps only the sign of a shifted sample, R-BUG-9): HIP encode
    byte-identical to the oracle, decode sample-identical, 5/3 lossless, also through windows."""
    import grok_amd as G
    from grok_amd.synth import synth_image
    img = synth_image(130, 150, 3, 8, 40 + roi[1]).astype(np.int32)
    kw = dict(numres=4, irreversible=irr, roi=roi, cblk_sty=0x40)
    cs = eng.encode(img, 8, params=G.default_params(numresolution=4, irreversible=irr, roi=roi, cblk_sty=0x40))
    ref = O.encode(img, 8, **kw)
    assert cs == ref
    dec = eng.decode(cs)
    np.testing.assert_array_equal(dec, O.decode(cs)[0])
    if not irr:
        np.testing.assert_array_equal(dec, img)
    win = (17, 9, 131, 120)
    np.testing.assert_array_equal(eng.decode_window(cs, win), O.decode(cs, partial=True)[0][:, 9:120, 17:131])


def test_roi_htj2k_mono16_tiles(eng):
    import grok_amd as G
    from grok_amd.synth import synth_image
    img = synth_image(200, 260, 1, 16, 77).astype(np.int32)
    cs = eng.encode(img, 16, params=G.default_params(roi=(0, 3), cblk_sty=0x40, tiles=(128, 96), tlm=True, plt=True))
    assert cs == O.encode(img, 16, roi=(0, 3), cblk_sty=0x40, tiles=(128, 96), tlm=True, plt=True)
    np.testing.assert_array_equal(eng.decode(cs), img)
