"""Known answers from Grok 9.2.0 itself for tiled rate control and odd-parity tiles.

The round-3 review ("What's weak" 1) ran Grok's own grk_compress on
synth_image(384, 520, 3, 8, 7) (grok_amd/synth.py, h=384, w=520) with the CLI flags below and
recorded the codestream sizes; these tests hold the oracle to them.  They pin:

  * the T2 simulation's budget arithmetic (T2Compress::compressPacketsSimulate,
    T2Compress.cpp:59-112 and :347-434, BitIO.cpp:35-52): a packet met with no byte left
    passes and the uint32 budget wraps, so the rest of the layer "fits" — the 8-px-wide edge
    tiles of -t 128,128 and -t 256,256 hit this, and Grok overshoots their budgets;
  * CodeStreamCompress::updateRates (:951-1027) with a TLM marker in the header size.

Grok is not rebuilt in this repository (its build is cmake with generated config headers:
DESIGN.md §4), so the review's numbers are the reference; sizes, not hashes, were recorded.
Cases the oracle does not yet reproduce are strict xfails naming the gap.
"""
import numpy as np
import pytest

import oracle as O
from grok_amd.synth import synth_image


@pytest.fixture(scope="module")
def img():
    return synth_image(384, 520, 3, 8, 7).astype(np.int32)


@pytest.mark.parametrize("flags,kw,grok_bytes", [
    ("-t 256,256 -r 20,5 -X", dict(tiles=(256, 256), layer_rate=[20.0, 5.0], tlm=True), 118560),
    ("-t 128,128 -r 30", dict(tiles=(128, 128), layer_rate=[30.0]), 22142),
])
def test_tiled_rate_control_equals_grok_size(img, flags, kw, grok_bytes):
    assert len(O.encode(img, 8, **kw)) == grok_bytes, flags


@pytest.mark.xfail(strict=True, reason="tile origins off the 2^5 grid (odd-parity DWT): the oracle is 1 byte "
                                       "short of Grok's 59,002 (58,945 before the parity-aware lifting)")
def test_odd_parity_tiles_rate_control_equals_grok_size(img):
    assert len(O.encode(img, 8, tiles=(200, 160), layer_rate=[30.0, 10.0])) == 59002


@pytest.mark.xfail(strict=True, reason="CPRL with precincts and a lossless last layer: the oracle is 20 bytes "
                                       "short of Grok's 430,903; cause not found")
def test_cprl_precincts_rate_control_equals_grok_size(img):
    kw = dict(prog_order="CPRL", precincts=[(64, 64), (32, 32)], layer_rate=[20.0, 5.0, 0.0])
    assert len(O.encode(img, 8, **kw)) == 430903


@pytest.mark.parametrize("tiles,numres", [((200, 160), 6), ((24, 40), 6), ((13, 7), 3), ((100, 70), 4)])
def test_odd_parity_tiles_lossless_round_trip(img, tiles, numres):
    # resolutions starting on odd coordinates take the odd ("cas1") lifting (WaveletFwd.cpp:486-489,
    # WaveletReverse.cpp:559-663): the 5/3 path stays lossless
    cs = O.encode(img, 8, tiles=tiles, numres=numres)
    dec, _ = O.decode(cs)
    np.testing.assert_array_equal(dec, img)
