"""Subsampled components on the HIP path (the oracle half, pinned by OpenJPEG, is
tests/test_subsampling.py): gk_encode with gk_set_subsampling writes the oracle's bytes, gk_decode
returns the oracle's planes (each component at its own size, host or device, int32 or 8/16-bit,
full or reduced resolution), and windows return each component's window on its grid."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
from subsampling_cases import CASES, engine_params, oracle_kw, planes

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


def _oracle_cs(name):
    W, H, sub, prec, kw = CASES[name]
    return O.encode(planes(name), prec, size=(W, H), **oracle_kw(name))


@pytest.mark.parametrize("name", sorted(CASES))
def test_engine_encode_equals_oracle(eng, name):
    import grok_amd as G
    W, H, sub, prec, kw = CASES[name]
    pk, origin = engine_params(name)
    cs = eng.encode(planes(name), prec, params=G.default_params(**pk), origin=origin, subsampling=sub, size=(W, H))
    assert cs == _oracle_cs(name)


@pytest.mark.parametrize("name", sorted(CASES))
def test_engine_decode_equals_oracle(eng, name):
    cs = _oracle_cs(name)
    want, _ = O.decode(cs)
    got = eng.decode(cs)
    assert len(got) == len(want)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("name", ["420_53", "tiled_rpcl_origin", "ht_420", "layers_97"])
def test_engine_decode_device(eng, name):
    import torch
    cs = _oracle_cs(name)
    want, _ = O.decode(cs)
    d = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    out = [torch.empty(w.shape, dtype=torch.int32, device="cuda") for w in want]
    eng.decode(d, len(cs), out=out)
    for o, w in zip(out, want):
        np.testing.assert_array_equal(o.cpu().numpy(), w)


def test_engine_decode_u8(eng):
    cs = _oracle_cs("420_53")
    want, _ = O.decode(cs)
    got = eng.decode(cs, sample_bytes=1)
    for g, w in zip(got, want):
        assert g.dtype == np.uint8
        np.testing.assert_array_equal(g.astype(np.int32), w)


@pytest.mark.parametrize("name", ["420_53_r6", "offset_odd", "tiled_pcrl", "422_97"])
@pytest.mark.parametrize("reduce", [1, 2])
def test_engine_decode_reduced(eng, name, reduce):
    cs = _oracle_cs(name)
    O.set_decode_reduce(reduce)
    try:
        want, _ = O.decode(cs)
    finally:
        O.set_decode_reduce(0)
    eng.set_decode_reduce(reduce)
    try:
        got = eng.decode(cs)
    finally:
        eng.set_decode_reduce(0)
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


def test_engine_round_trip_lossless(eng):
    import grok_amd as G
    name = "tiled_pcrl"
    W, H, sub, prec, kw = CASES[name]
    pk, origin = engine_params(name)
    src = planes(name)
    cs = eng.encode(src, prec, params=G.default_params(**pk), origin=origin, subsampling=sub, size=(W, H))
    for g, s in zip(eng.decode(cs), src):
        np.testing.assert_array_equal(g, s)


def _crop(planes, window, sub, origin, reduce=0):
    """Each component's window on its grid: canvas edges ceil(x / dx), then ceil(/ 2^reduce)."""
    x0, y0, x1, y1 = window
    X0, Y0 = origin
    cd = lambda a, b: -(-a // b)
    out = []
    for p, (dx, dy) in zip(planes, sub):
        gx = lambda v: cd(cd(v + X0, dx), 1 << reduce) - cd(cd(X0, dx), 1 << reduce)
        gy = lambda v: cd(cd(v + Y0, dy), 1 << reduce) - cd(cd(Y0, dy), 1 << reduce)
        out.append(p[gy(y0):gy(y1), gx(x0):gx(x1)])
    return out


WINDOWS = [(0, 0, 16, 16), (5, 3, 41, 37), (17, 11, 67, 45)]


@pytest.mark.parametrize("name", ["420_53", "offset_odd", "tiled_pcrl", "tiled_rpcl_origin", "422_97", "ht_420",
                                  "cprl_dx3"])
@pytest.mark.parametrize("wi", range(len(WINDOWS)))
def test_engine_subsampled_window(eng, name, wi):
    # Grok's window semantics: the composite's component c is the window's canvas rectangle on its
    # grid; a window decode takes the partial-tile inverse (the oracle's partial mode)
    W, H, sub, prec, kw = CASES[name]
    x0, y0, x1, y1 = WINDOWS[wi]
    win = (x0, y0, min(x1, W), min(y1, H))
    cs = _oracle_cs(name)
    full, _ = O.decode(cs, partial=True)
    origin = kw.get("origin") or kw.get("tile_origin") or (0, 0)
    got = eng.decode_window(cs, win)
    for g, w in zip(got, _crop(full, win, sub, origin)):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("name", ["420_53_r6", "tiled_pcrl", "422_97"])
def test_engine_subsampled_window_reduced(eng, name):
    W, H, sub, prec, kw = CASES[name]
    win = (5, 3, min(61, W), min(47, H))
    cs = _oracle_cs(name)
    O.set_decode_reduce(1)
    try:
        full, _ = O.decode(cs, partial=True)
    finally:
        O.set_decode_reduce(0)
    eng.set_decode_reduce(1)
    try:
        got = eng.decode_window(cs, win)
    finally:
        eng.set_decode_reduce(0)
    origin = kw.get("origin") or kw.get("tile_origin") or (0, 0)
    for g, w in zip(got, _crop(full, win, sub, origin, reduce=1)):
        np.testing.assert_array_equal(g, w)


def test_engine_tile_pitch_must_divide(eng):
    import grok_amd as G
    # a subsampling factor that does not divide the tile size gives irregular tile-components
    W, H = 64, 48
    sub = [(1, 1), (2, 2)]
    src = [np.zeros((48, 64), np.int32), np.zeros((24, 32), np.int32)]
    with pytest.raises(RuntimeError, match="does not divide the tile size"):
        eng.encode(src, 8, params=G.default_params(numresolution=2, tiles=(33, 48)), subsampling=sub, size=(W, H))


@pytest.mark.parametrize("name", ["tiled_pcrl", "tiled_rpcl_origin"])
def test_engine_subsampled_tile_ranges(eng, name):
    # gk_encode_tiles on a subsampled image (tile sharding): the header plus the parts of two tile
    # ranges assemble the whole-image stream
    import grok_amd as G
    W, H, sub, prec, kw = CASES[name]
    pk, origin = engine_params(name)
    params = G.default_params(**pk)
    src = planes(name)
    full = eng.encode(src, prec, params=params, origin=origin, subsampling=sub, size=(W, H))
    ntiles = -(-(W + (origin or (0, 0))[0]) // kw["tiles"][0]) * -(-(H + (origin or (0, 0))[1]) // kw["tiles"][1])
    k = ntiles // 2
    hdr, a, _ = eng.encode_tiles_subsampled(src, prec, 0, k, sub, (W, H), params=params, origin=origin)
    _, b, _ = eng.encode_tiles_subsampled(src, prec, k, ntiles, sub, (W, H), params=params, origin=origin)
    assert hdr + a + b + b"\xff\xd9" == full

