"""Code-block mode switches (GRK_CBLKSTY_LAZY/RESET/TERMALL/VSC/PTERM/SEGSYM, grok.h:98-103)
on the HIP path (gk_t1ms.hip + segment-aware T2) vs the oracle.

The mode combinations are those of the reference's own non-regression list
(tests/nonregression/test_suite.ctest.in:41,173-183: -M 1, 2, 4, 8, 16, 32, 5, 17, 20, 38)
plus all six together.  Parity unpinned against Grok itself: no reference-held fixture
carries a mode-switch codestream (the suite's input image is not in the repository), so
the bar is byte equality with the oracle's restatement of T1.cpp / mqc_enc.cpp /
T2Compress.cpp / T2Decompress.cpp, and lossless 5/3 round trips.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

MODES = [1, 2, 4, 8, 16, 32, 5, 17, 20, 38, 63]


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


def _img(seed, c, h, w, bits):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = (np.sin(xx / 7.0 + seed) * np.cos(yy / 5.0) + 1) * (1 << (bits - 2))
    img = base[None].repeat(c, 0) + rng.integers(0, 1 << (bits - 3), size=(c, h, w))
    return np.clip(img, 0, (1 << bits) - 1).astype(np.int32)


def _params(sty, irr=False, rates=None, numres=4, cblk=(32, 32), tiles=None):
    import grok_amd as G
    kw = dict(numresolution=numres, cblk=cblk, cblk_sty=sty, irreversible=irr)
    if rates:
        kw["layer_rate"] = rates
        kw["numlayers"] = len(rates)
    if tiles:
        kw["tiles"] = tiles
    return G.default_params(**kw)


@pytest.mark.parametrize("sty", MODES)
def test_modes_lossless_vs_oracle(eng, sty):
    img = _img(sty, 3, 97, 131, 8)
    cs = eng.encode(img, 8, params=_params(sty))
    ref = O.encode(img, 8, numres=4, cblk=(32, 32), cblk_sty=sty)
    assert cs == ref
    np.testing.assert_array_equal(eng.decode(ref), img)


@pytest.mark.parametrize("sty", MODES)
def test_modes_97_layers_vs_oracle(eng, sty):
    """9/7 with PCRD rate control: per-pass rates of terminated / raw passes feed the
    layer allocation, and layers cut codeword segments across packets."""
    img = _img(100 + sty, 3, 128, 96, 12)
    rates = [40, 20, 10]
    cs = eng.encode(img, 12, params=_params(sty, irr=True, rates=rates))
    ref = O.encode(img, 12, numres=4, cblk=(32, 32), cblk_sty=sty, irreversible=True, layer_rate=rates)
    assert cs == ref
    np.testing.assert_array_equal(eng.decode(ref), O.decode(ref)[0])


@pytest.mark.parametrize("sty", [1, 4, 5, 63])
def test_modes_lossless_layers_64(eng, sty):
    """5/3 with two rate-limited layers and 64x64 blocks of 16-bit samples (many bit-planes,
    so BYPASS reaches its raw passes), decoded from the truncated first layer too."""
    img = _img(200 + sty, 1, 160, 200, 16)
    rates = [20, 1]
    cs = eng.encode(img, 16, params=_params(sty, rates=rates, numres=5, cblk=(64, 64)))
    ref = O.encode(img, 16, numres=5, cblk=(64, 64), cblk_sty=sty, layer_rate=rates)
    assert cs == ref
    np.testing.assert_array_equal(eng.decode(ref), O.decode(ref)[0])


@pytest.mark.parametrize("sty", [5, 38])
def test_modes_tiled(eng, sty):
    img = _img(300 + sty, 3, 150, 170, 8)
    cs = eng.encode(img, 8, params=_params(sty, tiles=(64, 64)))
    ref = O.encode(img, 8, numres=4, cblk=(32, 32), cblk_sty=sty, tiles=(64, 64))
    assert cs == ref
    np.testing.assert_array_equal(eng.decode(cs), img)


def test_modes_ht_combination_refused(eng):
    img = _img(1, 1, 32, 32, 8)
    with pytest.raises(Exception):
        eng.encode(img, 8, params=_params(0x41))
