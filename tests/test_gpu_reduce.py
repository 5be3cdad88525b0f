"""Reduced-resolution decode (grk_decompress -r, grk_dparameters::cp_reduce): packets of the
discarded resolutions are skipped, the inverse DWT stops `reduce` levels early and the
output is ceil(size / 2^reduce).  HIP path (gk_set_decode_reduce) vs the oracle's same
reduction, sample-exact; the DC level of a flat image survives every reduction.  Parity
with Grok unpinned (no reference-held reduced decode)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.set_decode_reduce(0)
    e.close()


def _img(seed, c, h, w, bits=8):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = (np.sin(xx / 9.0 + seed) * np.cos(yy / 7.0) + 1) * (1 << (bits - 2))
    return np.clip(base[None].repeat(c, 0) + rng.integers(0, 1 << (bits - 3), size=(c, h, w)), 0,
                   (1 << bits) - 1).astype(np.int32)


CASES = [
    dict(c=3, h=150, w=170, kw=dict(numres=4)),
    dict(c=1, h=129, w=67, kw=dict(numres=5, irreversible=True), bits=12),
    dict(c=3, h=160, w=190, kw=dict(numres=4, tiles=(64, 96), plt=True)),
    dict(c=3, h=130, w=140, kw=dict(numres=4, irreversible=True, tiles=(64, 64))),
    dict(c=1, h=100, w=120, kw=dict(numres=3, cblk_sty=0x40)),
    dict(c=3, h=120, w=110, kw=dict(numres=4, prog_order="RPCL", precincts=[(32, 32)], layer_rate=[20, 5])),
]


def _gk(kw):
    import grok_amd as G
    k = dict(kw)
    k["numresolution"] = k.pop("numres")
    if "layer_rate" in k:
        k["numlayers"] = len(k["layer_rate"])
    return G.default_params(**k)


@pytest.mark.parametrize("ci", range(len(CASES)))
def test_reduce_vs_oracle(eng, ci):
    case = CASES[ci]
    bits = case.get("bits", 8)
    img = _img(ci, case["c"], case["h"], case["w"], bits)
    cs = eng.encode(img, bits, params=_gk(case["kw"]))
    try:
        for red in range(1, case["kw"]["numres"]):
            eng.set_decode_reduce(red)
            O.set_decode_reduce(red)
            dec = eng.decode(cs)
            ref = O.decode(cs)[0]
            f = 1 << red
            assert dec.shape == (case["c"], -(-case["h"] // f), -(-case["w"] // f))
            np.testing.assert_array_equal(dec, ref)
    finally:
        eng.set_decode_reduce(0)
        O.set_decode_reduce(0)
    np.testing.assert_array_equal(eng.decode(cs), O.decode(cs)[0])


def test_reduce_flat_level(eng):
    import grok_amd as G
    img = np.full((3, 96, 80), 137, np.int32)
    cs = eng.encode(img, 8, params=G.default_params(numresolution=5))
    try:
        for red in range(1, 5):
            eng.set_decode_reduce(red)
            assert (eng.decode(cs) == 137).all()
        eng.set_decode_reduce(5)
        with pytest.raises(Exception):
            eng.decode(cs)
    finally:
        eng.set_decode_reduce(0)


# reduced-resolution windows (grk_decompress -r n -d x0,y0,x1,y1): the window is given at full
# resolution and returned on the reduced canvas, every edge ceil(x / 2^n) (the composite
# component bounds, CodeStreamDecompress.cpp:471-481); the samples are the oracle's reduced
# decode under the partial-tile rule a window selects (WaveletReverse.cpp:1551-1554), cropped
WINDOWS = [(0, 0, 37, 41), (13, 7, 101, 66), (33, 29, 34, 30), (5, 50, 170, 150), (64, 0, 128, 64)]


@pytest.mark.parametrize("ci", [0, 1, 2, 3, 5])
def test_reduce_window_vs_oracle(eng, ci):
    case = CASES[ci]
    bits = case.get("bits", 8)
    img = _img(ci, case["c"], case["h"], case["w"], bits)
    cs = eng.encode(img, bits, params=_gk(case["kw"]))
    cd = lambda v, r: -(-v >> r)
    try:
        for red in range(1, case["kw"]["numres"]):
            eng.set_decode_reduce(red)
            O.set_decode_reduce(red)
            ref = O.decode(cs, partial=True)[0]
            for (x0, y0, x1, y1) in WINDOWS:
                x1, y1 = min(x1, case["w"]), min(y1, case["h"])
                if x0 >= x1 or y0 >= y1:
                    continue
                qx0, qy0, qx1, qy1 = cd(x0, red), cd(y0, red), cd(x1, red), cd(y1, red)
                if qx0 >= qx1 or qy0 >= qy1:
                    continue   # (nothing left at this reduction)
                dec = eng.decode_window(cs, (x0, y0, x1, y1))
                assert dec.shape == (case["c"], qy1 - qy0, qx1 - qx0)
                np.testing.assert_array_equal(dec, ref[:, qy0:qy1, qx0:qx1], err_msg=f"red {red} window {(x0, y0, x1, y1)}")
    finally:
        eng.set_decode_reduce(0)
        O.set_decode_reduce(0)
