"""Main-header COC on the HIP path (the oracle half, pinned by OpenJPEG, is tests/test_coc.py):
components with their own decomposition levels, code-block size and style (Part-1, mode switches,
HT, wide blocks), transform and precincts decode to the oracle's planes, i.e. to each
component's own single-component decode; full and reduced, host and device streams, windows."""
import numpy as np
import pytest

import oracle as O
from test_coc import CASES, single_decodes, stream

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("name", sorted(CASES))
def test_engine_coc_equals_oracle(eng, name):
    cs = stream(name)
    want, _ = O.decode(cs)
    got = eng.decode(cs)
    for g, w, s in zip(got, want, single_decodes(name)):
        np.testing.assert_array_equal(g, w)
        np.testing.assert_array_equal(g, s)


@pytest.mark.parametrize("name", ["levels_cblk_97_prc", "ht_and_part1", "mode_switches"])
def test_engine_coc_device_stream(eng, name):
    import torch
    cs = stream(name)
    want, _ = O.decode(cs)
    d = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    got = eng.decode(d, len(cs))
    for g, w in zip(got, want):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("name", ["levels_cblk_97_prc", "ht_and_part1", "layers_rate"])
def test_engine_coc_reduced(eng, name):
    cs = stream(name)
    eng.set_decode_reduce(1)
    try:
        got = eng.decode(cs)
    finally:
        eng.set_decode_reduce(0)
    for g, w in zip(got, single_decodes(name, reduce=1)):
        np.testing.assert_array_equal(g, w)


@pytest.mark.parametrize("name", ["levels_cblk_97_prc", "ht_and_part1", "mode_switches", "wide_block"])
@pytest.mark.parametrize("win", [(0, 0, 16, 16), (7, 5, 45, 39), (33, 21, 60, 50)])
def test_engine_coc_window(eng, name, win):
    # each component's window equals the crop of the oracle's partial-rule decode (its own levels,
    # code-blocks and transform project the window onto its bands)
    cs = stream(name)
    full, _ = O.decode(cs, partial=True)
    x0, y0, x1, y1 = win
    got = eng.decode_window(cs, win)
    for g, f in zip(got, full):
        np.testing.assert_array_equal(g, f[y0:y1, x0:x1])
