"""HTJ2K block coder on the HIP path (k_ht_enc / k_ht_dec) vs Grok and the oracle.

Bar: HT codestreams byte-identical to Grok's
(`grk_compress -M 64`), decodes sample-exact (HT here is reversible 5/3 only).
Cases: Grok's HT fixtures, seeded random shapes / code-block sizes / depths
against the oracle (which is itself pinned to the fixtures), ragged and
degenerate shapes, constant and extreme images, signed input, corrupt input,
and switching the same engine between Part-1 and HT plans.
"""
import numpy as np
import pytest

from conftest import FIXTURES, fixture_ids
import oracle as O

pytestmark = pytest.mark.gpu

HT = [f for f in FIXTURES if f.ht and not f.tiled]
HT_ALL = [f for f in FIXTURES if f.ht]


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


def ht_params(numres=6, cblk=(64, 64)):
    import grok_amd as G
    return G.default_params(numresolution=numres, cblk=cblk, cblk_sty=0x40)


@pytest.mark.parametrize("fx", HT_ALL, ids=fixture_ids(HT_ALL))
def test_ht_encode_bit_exact_vs_grok(eng, fx):
    from test_gpu_parity import gk_params
    cs = eng.encode(fx.img, fx.bits, params=gk_params(fx.kw))
    assert len(cs) == len(fx.cs)
    assert cs == fx.cs


@pytest.mark.parametrize("fx", HT_ALL, ids=fixture_ids(HT_ALL))
def test_ht_decode_grok_stream(eng, fx):
    np.testing.assert_array_equal(eng.decode(fx.cs), fx.grok_decoded)
    np.testing.assert_array_equal(eng.decode(fx.cs), fx.img)


def _case(seed):
    rng = np.random.default_rng(5000 + seed)
    c = int(rng.choice([1, 3]))
    bits = int(rng.choice([8, 10, 12, 16]))
    h, w = int(rng.integers(1, 600)), int(rng.integers(1, 600))
    cb = [(64, 64), (32, 32), (64, 16), (16, 64), (8, 8), (4, 4), (64, 4), (4, 64)][seed % 8]
    numres = int(rng.integers(1, 8))
    kind = seed % 3
    if kind == 0:
        img = rng.integers(0, 1 << bits, size=(c, h, w))
    elif kind == 1:   # smooth + noise: many small magnitudes, MEL runs
        yy, xx = np.mgrid[0:h, 0:w]
        base = ((np.sin(xx / 23.0) + np.cos(yy / 17.0)) * 0.2 + 0.5) * ((1 << bits) - 1)
        img = np.clip(base[None] + rng.normal(0, 2, size=(c, h, w)), 0, (1 << bits) - 1)
    else:             # sparse: mostly flat with rare spikes (long zero runs, large u)
        img = np.full((c, h, w), 1 << (bits - 1))
        m = rng.random((c, h, w)) < 0.01
        img[m] = rng.integers(0, 1 << bits, size=int(m.sum()))
    return img.astype(np.int32), bits, numres, cb


@pytest.mark.parametrize("seed", range(24))
def test_ht_random_vs_oracle(eng, seed):
    img, bits, numres, cb = _case(seed)
    ref = O.encode(img, bits, numres=numres, cblk=cb, cblk_sty=64)
    cs = eng.encode(img, bits, params=ht_params(numres, cb))
    assert cs == ref
    np.testing.assert_array_equal(eng.decode(cs), img)


@pytest.mark.parametrize("shape", [(1, 1, 1), (1, 1, 513), (1, 257, 1), (3, 2, 2), (1, 3, 5), (3, 65, 67),
                                   (1, 128, 130)])
def test_ht_edge_shapes(eng, shape):
    rng = np.random.default_rng(sum(shape))
    img = rng.integers(0, 256, size=shape).astype(np.int32)
    ref = O.encode(img, 8, numres=3, cblk=(64, 64), cblk_sty=64)
    cs = eng.encode(img, 8, params=ht_params(3))
    assert cs == ref
    np.testing.assert_array_equal(eng.decode(cs), img)


@pytest.mark.parametrize("value", [0, 255, 128])
def test_ht_constant(eng, value):
    img = np.full((3, 100, 90), value, np.int32)
    cs = eng.encode(img, 8, params=ht_params())
    assert cs == O.encode(img, 8, cblk_sty=64)
    np.testing.assert_array_equal(eng.decode(cs), img)


def test_ht_extremes_16bit(eng):
    # alternating 0 / 65535: the largest magnitudes the 16-bit HT QCD admits
    img = np.zeros((1, 96, 96), np.int32)
    img[0, ::2, 1::2] = 65535
    img[0, 1::2, ::2] = 65535
    cs = eng.encode(img, 16, params=ht_params())
    assert cs == O.encode(img, 16, cblk_sty=64)
    np.testing.assert_array_equal(eng.decode(cs), img)


def test_ht_signed(eng):
    rng = np.random.default_rng(9)
    img = rng.integers(-2048, 2048, size=(1, 77, 91)).astype(np.int32)
    cs = eng.encode(img, 12, signed=True, params=ht_params(4))
    assert cs == O.encode(img, 12, signed=True, numres=4, cblk_sty=64)
    np.testing.assert_array_equal(eng.decode(cs), img)


def test_ht_and_part1_same_engine(eng):
    # plan cache keyed on the block-coder style: alternate HT / Part-1 / HT
    fx = HT[0]
    a = eng.encode(fx.img, fx.bits, params=ht_params())
    import grok_amd as G
    b = eng.encode(fx.img, fx.bits, params=G.default_params())
    c = eng.encode(fx.img, fx.bits, params=ht_params())
    assert a == fx.cs and c == fx.cs and b != a
    np.testing.assert_array_equal(eng.decode(b), fx.img)
    np.testing.assert_array_equal(eng.decode(a), fx.img)


def test_ht_corrupt_stream_reports_error(eng):
    fx = HT[0]
    bad = bytearray(fx.cs)
    # clobber the last bytes of the tile body (Scup of the final code-blocks)
    for i in range(len(bad) - 40, len(bad) - 2):
        bad[i] = 0xFF
    with pytest.raises(RuntimeError):
        eng.decode(bytes(bad))
    # the engine is still usable afterwards
    np.testing.assert_array_equal(eng.decode(fx.cs), fx.img)
