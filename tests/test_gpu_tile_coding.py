"""Tiles coded with their own parameters (tile-part COD / COC / QCD / QCC) on the HIP path; the
oracle half, pinned by OpenJPEG, is tests/test_tile_coding.py.  The engine decodes the tiles with
the main header's coding in one pass and every other tile in a pass of its own (its plan and
quantisation), into one output: full and reduced, host and device (TLM-located) streams, 8-bit
output, windows across tiles of both kinds, and Grok's whole-tile rule for a tile decode."""
import numpy as np
import pytest

import oracle as O
from tile_coding import CASES, expected, stream, tile_rects

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("name", sorted(CASES))
def test_engine_tile_coding(eng, name):
    cs = stream(name)
    want = expected(name)
    np.testing.assert_array_equal(O.decode(cs)[0], want)
    np.testing.assert_array_equal(eng.decode(cs), want)


@pytest.mark.parametrize("name", ["levels_cblk", "coc_form", "prog_layers_sop", "scope_irrev"])
def test_engine_tile_coding_device_tlm(eng, name):
    import torch
    cs = stream(name, tlm=True)
    d = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    np.testing.assert_array_equal(eng.decode(d, len(cs)), expected(name))


@pytest.mark.parametrize("name", ["levels_cblk", "rev_to_irrev", "coc_form", "ht_tile", "ragged_tiles", "origin_tiles"])
def test_engine_tile_coding_reduced(eng, name):
    eng.set_decode_reduce(1)
    try:
        got = eng.decode(stream(name))
    finally:
        eng.set_decode_reduce(0)
    np.testing.assert_array_equal(got, expected(name, reduce=1))


def test_engine_tile_coding_u8(eng):
    got = eng.decode(stream("ht_tile"), sample_bytes=1)
    assert got.dtype == np.uint8
    np.testing.assert_array_equal(got.astype(np.int32), expected("ht_tile"))


@pytest.mark.parametrize("name", ["levels_cblk", "rev_to_irrev", "modes_tile", "ragged_tiles", "origin_tiles"])
@pytest.mark.parametrize("win", [(5, 7, 61, 50), (40, 30, 60, 45), (0, 0, 20, 20)])
def test_engine_tile_coding_window(eng, name, win):
    H, W = CASES[name][:2]
    x0, y0, x1, y1 = win
    x1, y1 = min(x1, W), min(y1, H)
    want = expected(name, partial=True)[:, y0:y1, x0:x1]
    np.testing.assert_array_equal(eng.decode_window(stream(name), (x0, y0, x1, y1)), want)


@pytest.mark.parametrize("name", ["levels_cblk", "scope_irrev"])
def test_engine_tile_coding_tile_decode(eng, name):
    # -tile t without a window: Grok's whole-tile rule, each tile (B or A coded) on its own
    cs = stream(name)
    want = expected(name)
    eng.set_window_rule(True)
    try:
        for t, (x0, y0, x1, y1) in tile_rects(name).items():
            got = eng.decode_window(cs, (x0, y0, x1, y1))
            np.testing.assert_array_equal(got, want[:, y0:y1, x0:x1], err_msg=f"tile {t}")
    finally:
        eng.set_window_rule(False)


def test_engine_tile_coding_reduce_past_a_tile_refused(eng):
    eng.set_decode_reduce(2)
    try:
        with pytest.raises(RuntimeError, match="reduce must be less"):
            eng.decode(stream("ragged_tiles"))
    finally:
        eng.set_decode_reduce(0)


@pytest.mark.parametrize("reduce", [0, 1])
def test_engine_tile_coding_device_output(eng, reduce):
    # the passes write straight into the caller's device planes
    import torch
    name = "levels_cblk"
    want = expected(name, reduce=reduce)
    out = torch.full(want.shape, -1, dtype=torch.int32, device="cuda")
    eng.set_decode_reduce(reduce)
    try:
        eng.decode(stream(name), out=out)
    finally:
        eng.set_decode_reduce(0)
    np.testing.assert_array_equal(out.cpu().numpy(), want)


def test_engine_tile_coding_subsampled():
    # a 4:2:0 stream whose tile 1 is coded with its own levels and code-blocks
    import grok_amd as G
    import tile_coding as TC
    from subsampling_cases import comp_shape
    W, H, sub = 96, 80, [(1, 1), (2, 2), (2, 2)]
    rng = np.random.default_rng(5)
    src = [rng.integers(0, 256, size=comp_shape(W, H, dx, dy)).astype(np.int32) for dx, dy in sub]
    a = O.encode(src, 8, size=(W, H), subsampling=sub, tiles=TC.TILES, numres=3)
    b = O.encode(src, 8, size=(W, H), subsampling=sub, tiles=TC.TILES, numres=2, cblk=(16, 16))
    cs = TC.splice(a, b, {1}, "cod")
    want, _ = O.decode(cs)
    e = G.Engine(0)
    try:
        got = e.decode(cs)
    finally:
        e.close()
    for g, w, s in zip(got, want, src):
        np.testing.assert_array_equal(g, w)
        np.testing.assert_array_equal(g, s)   # (lossless either way)


@pytest.mark.parametrize("name", ["ht_and_part1", "mode_switches", "wide_block"])
def test_engine_tile_cod_resets_main_coc(eng, name):
    import j2k_markers as J
    import test_coc
    cs = test_coc.stream(name)
    t = J.insert_tile_part(cs, J.cod(cs))
    for g, w in zip(eng.decode(t), O.decode(t)[0]):
        np.testing.assert_array_equal(g, w)
