"""Multi-tile images on the HIP path (batched per-tile DWT, all tiles' code-blocks
in one T1 launch, per-tile T2, SOT/TLM/PLT) vs Grok and the oracle.

Bar: codestreams byte-identical to
Grok's `-t W,H [-X] [-L]` output (fixtures) and to the oracle on seeded random
tilings (ragged edge tiles, 1-tile-wide strips, Part 1 and HT, TLM/PLT on and
off); decodes sample-exact.  Tile sizes are multiples of 2^(levels) (tile DWT
parity 0), which covers the C4/C5 configurations (1024 x 1024 tiles).
"""
import numpy as np
import pytest

from conftest import FIXTURES, fixture_ids
import oracle as O

pytestmark = pytest.mark.gpu

TILED = [f for f in FIXTURES if f.tiled]


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


def _params(**kw):
    import grok_amd as G
    numres = kw.pop("numres", 6)
    return G.default_params(numresolution=numres, **kw)


@pytest.mark.parametrize("fx", TILED, ids=fixture_ids(TILED))
def test_tiled_fixture_encode_bit_exact(eng, fx):
    from test_gpu_parity import gk_params
    cs = eng.encode(fx.img, fx.bits, params=gk_params(fx.kw))
    assert cs == fx.cs


@pytest.mark.parametrize("fx", TILED, ids=fixture_ids(TILED))
def test_tiled_fixture_decode(eng, fx):
    dec = eng.decode(fx.cs)
    if fx.lossless:
        np.testing.assert_array_equal(dec, fx.img)
    else:
        assert np.abs(dec.astype(np.int64) - fx.grok_decoded).max() <= 1


@pytest.mark.parametrize("seed", range(16))
def test_tiled_random_vs_oracle(eng, seed):
    rng = np.random.default_rng(700 + seed)
    numres = int(rng.integers(1, 7))
    unit = 1 << (numres - 1)
    tw = unit * int(rng.integers(1, max(2, 256 // unit) + 1))
    th = unit * int(rng.integers(1, max(2, 256 // unit) + 1))
    w, h = int(rng.integers(1, 3 * tw + 5)), int(rng.integers(1, 3 * th + 5))
    c = int(rng.choice([1, 3]))
    bits = int(rng.choice([8, 12, 16]))
    ht = bool(seed % 2)
    tlm, plt = bool(seed % 3 == 0), bool(seed % 4 < 2)
    cb = [(64, 64), (32, 32), (16, 64)][seed % 3]
    img = rng.integers(0, 1 << bits, size=(c, h, w)).astype(np.int32)
    kw = dict(numres=numres, cblk=cb, tiles=(tw, th), tlm=tlm, plt=plt, cblk_sty=64 if ht else 0)
    ref = O.encode(img, bits, **kw)
    gkw = dict(kw)
    gkw["numres"] = gkw["numres"]
    cs = eng.encode(img, bits, params=_params(**gkw))
    assert cs == ref, (w, h, tw, th, numres, ht)
    np.testing.assert_array_equal(eng.decode(cs), img)


def test_tiled_97(eng):
    rng = np.random.default_rng(5)
    img = rng.integers(0, 4096, size=(3, 200, 260)).astype(np.int32)
    kw = dict(tiles=(128, 64), irreversible=True, tlm=True, plt=True)
    ref = O.encode(img, 12, **kw)
    cs = eng.encode(img, 12, params=_params(**kw))
    assert cs == ref
    dec_o, _ = O.decode(cs)
    assert np.abs(eng.decode(cs).astype(np.int64) - dec_o).max() <= 1


def test_tile_grid_rules(eng):
    # tile sizes off the 2^levels grid are refused (the tile DWT would need odd parity)
    img = np.zeros((1, 100, 100), np.int32)
    with pytest.raises(RuntimeError):
        eng.encode(img, 8, params=_params(tiles=(48, 48)))
    # a tile larger than the image is a single tile
    cs = eng.encode(img, 8, params=_params(tiles=(4096, 4096)))
    np.testing.assert_array_equal(eng.decode(cs), img)


def test_engine_reuse_refreshes_params(eng):
    # same geometry, different non-geometric parameters (TLM/PLT, layer rates): the
    # cached plan must not carry the previous call's settings over
    rng = np.random.default_rng(77)
    img = rng.integers(0, 256, size=(3, 256, 256)).astype(np.int32)
    for kw in (dict(tiles=(128, 128)), dict(tiles=(128, 128), tlm=True, plt=True), dict(tiles=(128, 128))):
        assert eng.encode(img, 8, params=_params(**kw)) == O.encode(img, 8, **kw)
    for rates in ([40.0, 20.0], [20.0, 10.0], [40.0, 20.0]):
        kw = dict(irreversible=True, layer_rate=rates)
        assert eng.encode(img, 8, params=_params(**kw)) == O.encode(img, 8, **kw)
