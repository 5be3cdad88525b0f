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
