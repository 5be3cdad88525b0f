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


@pytest.mark.parametrize("fx", PART1, ids=fixture_ids(PART1))
def test_oracle_decode_matches_grok(fx):
    dec, prec = O.decode(fx.cs)
    assert prec == fx.bits
    assert dec.shape == fx.grok_decoded.shape
    np.testing.assert_array_equal(dec, fx.grok_decoded)


@pytest.mark.parametrize("fx", PART1_LOSSLESS, ids=fixture_ids(PART1_LOSSLESS))
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
