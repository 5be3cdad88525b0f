"""Image and tile-grid offsets on the HIP path (SIZ XOsiz / YOsiz / XTOsiz / YTOsiz; grk_compress
-d x0,y0 and -T x0,y0; B.2-B.3).

The image area sits at (x0, y0) on the canvas and the tile grid at (tx0, ty0) <= (x0, y0): tile
rectangles, resolution and band geometry are canvas coordinates (so the lifting parity follows
the canvas position, WaveletFwd.cpp:486-489), work planes hold the image area.  Bar: codestreams
byte-identical to the oracle (which restates B.2-B.3 with its odd-parity lifting; Grok fixtures
with offsets do not exist, so these cases are parity-unpinned against Grok itself beyond the
oracle's lossless round trips), decodes equal to the oracle's, 5/3 lossless, windows and reduced
decodes relative to the image origin.
"""
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


def _img(h, w, c, bits, seed):
    from grok_amd.synth import synth_image
    return synth_image(h, w, c, bits, seed).astype(np.int32)


CASES = [
    # (h, w, c, bits), origin, tile_origin, tiles, extra
    ((90, 110, 3, 8), (3, 5), None, None, {}),
    ((90, 110, 3, 8), (17, 9), (5, 2), (32, 48), {}),
    ((90, 110, 3, 8), (1, 1), None, (13, 7), dict(numres=3)),
    ((90, 110, 3, 8), (100, 200), (90, 150), (64, 64), {}),
    ((90, 110, 3, 8), None, (7, 3), (40, 40), {}),
    ((120, 100, 3, 12), (33, 21), (31, 20), (64, 32), dict(irreversible=True)),
    ((100, 96, 1, 16), (5, 6), (0, 0), (48, 40), dict(cblk_sty=64)),
    ((97, 113, 3, 8), (65, 33), (64, 32), (32, 32), dict(tlm=True, plt=True, prog_order="RPCL")),
]


def _encode(eng, img, bits, origin, tile_origin, tiles, extra):
    import grok_amd as G
    kw = dict(extra)
    nr = kw.pop("numres", 6)
    p = G.default_params(numresolution=nr, tiles=tiles, tile_origin=tile_origin, **kw)
    cs = eng.encode(img, bits, params=p, origin=origin)
    ref = O.encode(img, bits, numres=nr, tiles=tiles, origin=origin, tile_origin=tile_origin, **kw)
    return cs, ref


@pytest.mark.parametrize("i", range(len(CASES)))
def test_offsets_vs_oracle(eng, i):
    (h, w, c, bits), origin, tile_origin, tiles, extra = CASES[i]
    img = _img(h, w, c, bits, 50 + i)
    cs, ref = _encode(eng, img, bits, origin, tile_origin, tiles, extra)
    assert cs == ref, CASES[i]
    info = eng.read_header(cs)
    ox, oy = origin if origin else (tile_origin if tile_origin else (0, 0))
    assert (info.x0, info.y0, info.w, info.h) == (ox, oy, w, h)
    want, _ = O.decode(cs)
    got = eng.decode(cs)
    if extra.get("irreversible"):
        assert np.abs(got.astype(np.int64) - want).max() <= 1
    else:
        np.testing.assert_array_equal(got, img)
        np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("red", [1, 2, 3])
def test_offsets_reduce(eng, red):
    img = _img(90, 110, 3, 8, 61)
    cs = O.encode(img, 8, tiles=(32, 48), origin=(17, 9), tile_origin=(5, 2))
    O.set_decode_reduce(red)
    try:
        want, _ = O.decode(cs)
    finally:
        O.set_decode_reduce(0)
    eng.set_decode_reduce(red)
    try:
        got = eng.decode(cs)
    finally:
        eng.set_decode_reduce(0)
    assert got.shape == want.shape
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize("win", [(0, 0, 110, 90), (10, 20, 60, 70), (0, 0, 1, 1), (100, 80, 110, 90)])
def test_offsets_window(eng, win):
    img = _img(90, 110, 3, 8, 62)
    cs = O.encode(img, 8, tiles=(32, 48), origin=(17, 9), tile_origin=(5, 2), tlm=True, plt=True)
    x0, y0, x1, y1 = win
    np.testing.assert_array_equal(eng.decode_window(cs, win), img[:, y0:y1, x0:x1])


def test_offsets_refused(eng):
    import grok_amd as G
    img = _img(40, 40, 1, 8, 63)
    with pytest.raises(RuntimeError, match="tile grid origin"):
        eng.encode(img, 8, params=G.default_params(tiles=(16, 16), tile_origin=(9, 9)), origin=(5, 5))
    with pytest.raises(RuntimeError, match="first tile"):
        eng.encode(img, 8, params=G.default_params(tiles=(16, 16), tile_origin=(0, 0)), origin=(20, 20))


def test_window_takes_partial_inverse_rule(eng):
    # A tile one column wide on an odd canvas coordinate (image origin x 63, 64-wide tiles) has a
    # single odd sample across at its top resolution.  Grok decodes through a window with its
    # partial-tile inverse (S >>= 1) and without one with bandH / 2; the engine follows
    # (ctx->dwt_partial) and so does the oracle (decode(partial=True)); the two can differ only
    # on a negative odd coefficient of a lossy stream, so both rules are also checked directly
    # (test_grok_defects.py::test_single_odd_sample_rule)
    import grok_amd as G
    img = _img(90, 110, 3, 8, 77)
    kw = dict(tiles=(64, 64), layer_rate=[3.0])
    p = G.default_params(tiles=(64, 64), numlayers=1, layer_rate=[3.0])
    cs = eng.encode(img, 8, params=p, origin=(63, 0))
    assert cs == O.encode(img, 8, origin=(63, 0), **kw)
    whole, _ = O.decode(cs)
    part, _ = O.decode(cs, partial=True)
    np.testing.assert_array_equal(eng.decode(cs), whole)
    win = (0, 5, 40, 80)
    np.testing.assert_array_equal(eng.decode_window(cs, win), part[:, win[1]:win[3], win[0]:win[2]])
