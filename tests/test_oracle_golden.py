"""Pin the CPU oracle (oracle/j2k_oracle.cpp) against reference Grok 9.2.0.

The fixtures in tests/golden/ hold Grok's own codestreams and decodes of small
seeded images (tests/golden/make_fixtures.py).  The oracle must reproduce
Grok's 5/3 codestreams byte for byte and Grok's decodes sample for sample
before it is trusted as the checker for the HIP path.
"""
import numpy as np
import pytest

from conftest import FIXTURES, fixture_ids
import oracle as O

PART1 = [f for f in FIXTURES if not f.ht]
HT = [f for f in FIXTURES if f.ht]
PART1_LOSSLESS = [f for f in PART1 if f.lossless]
PART1_LOSSY = [f for f in PART1 if not f.lossless]


def oracle_kw(kw):
    k = dict(kw)
    k.pop("cblk_sty", None)
    return k


@pytest.mark.parametrize("fx", PART1_LOSSLESS, ids=fixture_ids(PART1_LOSSLESS))
def test_oracle_encode_matches_grok(fx):
    cs = O.encode(fx.img, fx.bits, **oracle_kw(fx.kw))
    assert len(cs) == len(fx.cs)
    assert cs == fx.cs


@pytest.mark.parametrize("fx", PART1_LOSSY, ids=fixture_ids(PART1_LOSSY))
def test_oracle_encode_97_matches_grok(fx):
    # 9/7 + ICT, with and without PCRD rate allocation (-r 40,20,10): Grok's float
    # lifting order reproduced exactly, so the codestream is byte-identical
    cs = O.encode(fx.img, fx.bits, **oracle_kw(fx.kw))
    assert cs == fx.cs


@pytest.mark.parametrize("fx", HT, ids=fixture_ids(HT))
def test_oracle_encode_ht_matches_grok(fx):
    # HTJ2K (-M 64): Rsiz 0x4000, CAP, HT reversible QCD (BIBO gains, 1 guard
    # bit), one cleanup pass per block (MEL / VLC / MagSgn) — byte-identical
    cs = O.encode(fx.img, fx.bits, **fx.kw)
    assert cs == fx.cs


@pytest.mark.parametrize("fx", FIXTURES, ids=fixture_ids(FIXTURES))
def test_oracle_decode_matches_grok(fx):
    dec, prec = O.decode(fx.cs)
    assert prec == fx.bits
    assert dec.shape == fx.grok_decoded.shape
    np.testing.assert_array_equal(dec, fx.grok_decoded)


@pytest.mark.parametrize("fx", [f for f in FIXTURES if f.lossless], ids=fixture_ids([f for f in FIXTURES if f.lossless]))
def test_grok_lossless_round_trip(fx):
    # the fixtures themselves: Grok's 5/3 decode reproduces the source
    np.testing.assert_array_equal(fx.grok_decoded, fx.img)


def test_oracle_t1_block_round_trip():
    rng = np.random.default_rng(7)
    for (h, w) in [(64, 64), (1, 1), (3, 64), (64, 5), (17, 33)]:
        for orient in range(4):
            coef = rng.integers(-3000, 3000, size=(h, w)).astype(np.int32)
            coef[rng.random((h, w)) < 0.4] = 0
            data, nbps, npass, rates, lens = O.t1_encode_cblk(coef, orient)
            assert npass == (3 * nbps - 2 if nbps else 0)
            dec = O.t1_decode_cblk(data, npass, nbps, orient, w, h)
            # decoded value is Grok's pre-filter magnitude (2M+1)<<(q-1); ShiftFilter
            # (filters/PostDecompressFilters.h) halves it with C truncation -> exact coefficient
            np.testing.assert_array_equal(np.fix(dec / 2).astype(np.int32), coef)


def test_oracle_ht_block_round_trip():
    # HT cleanup pass: encode -> decode is the identity on signed coefficients,
    # over ragged shapes (odd widths/heights, 1-row/1-column blocks), sparse
    # blocks (MEL runs), dense large magnitudes (U-VLC suffixes, u > 2 pairs)
    # and all-zero blocks
    rng = np.random.default_rng(11)
    shapes = [(64, 64), (1, 1), (1, 64), (64, 1), (2, 3), (3, 2), (5, 7), (17, 33), (32, 128), (4, 1024)]
    for (h, w) in shapes:
        for mag, dens in [(1, 0.05), (7, 0.3), (3000, 0.6), (1 << 20, 1.0), (0, 0.0)]:
            coef = rng.integers(-mag, mag + 1, size=(h, w)).astype(np.int32)
            coef[rng.random((h, w)) >= dens] = 0
            data = O.ht_encode_cblk(coef)
            np.testing.assert_array_equal(O.ht_decode_cblk(data, w, h), coef)


@pytest.mark.parametrize("seed", range(6))
def test_oracle_ht_codestream_round_trip(seed):
    rng = np.random.default_rng(100 + seed)
    h, w = int(rng.integers(1, 90)), int(rng.integers(1, 90))
    nc = int(rng.choice([1, 3]))
    bits = int(rng.choice([8, 12, 16]))
    cb = [(64, 64), (32, 32), (16, 64), (64, 4), (8, 8)][seed % 5]
    img = rng.integers(0, 1 << bits, size=(nc, h, w)).astype(np.int32)
    cs = O.encode(img, bits, numres=int(rng.integers(1, 6)), cblk=cb, cblk_sty=64)
    dec, prec = O.decode(cs)
    assert prec == bits
    np.testing.assert_array_equal(dec, img)
