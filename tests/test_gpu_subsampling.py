"""Subsampled components on the HIP path (the oracle half, pinned by OpenJPEG, is
tests/test_subsampling.py): gk_encode with gk_set_subsampling writes the oracle's bytes, gk_decode
returns the oracle's planes (each component at its own size, host or device, int32 or 8/16-bit,
full or reduced resolution), and windows of such streams are refused."""
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


def test_engine_subsampled_window_refused(eng):
    cs = _oracle_cs("420_53")
    with pytest.raises(RuntimeError, match="window decodes of subsampled"):
        eng.decode_window(cs, (0, 0, 16, 16))


def test_engine_tile_pitch_must_divide(eng):
    import grok_amd as G
    # a subsampling factor that does not divide the tile size gives irregular tile-components
    W, H = 64, 48
    sub = [(1, 1), (2, 2)]
    src = [np.zeros((48, 64), np.int32), np.zeros((24, 32), np.int32)]
    with pytest.raises(RuntimeError, match="does not divide the tile size"):
        eng.encode(src, 8, params=G.default_params(numresolution=2, tiles=(33, 48)), subsampling=sub, size=(W, H))
