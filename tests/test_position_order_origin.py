"""Position-driven progressions (RPCL / PCRL / CPRL) on an image whose origin is off the precinct
grid.  Grok's walk (PacketIter::generatePrecinctIndex, PacketIter.cpp:287-335) emits the first
precinct of a resolution at the tile origin only when the resolution starts off its precinct grid;
a resolution that starts on it (e.g. origin 3, level 1: resolution origin 2, precincts of 2) waits
for the canvas position 2^(PPx + level) * index, after the precincts the tile origin emits.
OpenJPEG 2.5.4's iterator (opj_pi_next_*) has the same rule, so it decodes the oracle's streams
losslessly (CPU); the engine orders packets by those positions and writes / reads the oracle's
bytes (GPU)."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
import openjpeg

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

# (origin, precincts, numres, tiles)
CASES = [
    ((3, 5), [(4, 4), (2, 2)], 3, None),
    ((1, 1), [(8, 8), (4, 4), (2, 2)], 4, None),
    ((5, 3), [(16, 16), (8, 8)], 3, (40, 24)),
]


def _img(seed, h, w):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 256, size=(3, h, w)).astype(np.int32)


def _okw(ci, prog):
    origin, prc, numres, tiles = CASES[ci]
    kw = dict(numres=numres, cblk=(4, 4), precincts=prc, prog_order=prog, origin=origin)
    if tiles:
        kw.update(tiles=tiles, tile_origin=(0, 0))
    return kw


@pytest.mark.skipif(not openjpeg.available(), reason="libopenjp2 (Pillow's) not present")
@pytest.mark.parametrize("prog", ["RPCL", "PCRL", "CPRL"])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_oracle_off_grid_origin_equals_openjpeg(ci, prog):
    img = _img(ci, 37, 45)
    cs = O.encode(img, 8, **_okw(ci, prog))
    for (dx, dy, a), src in zip(openjpeg.decode(cs), img):
        np.testing.assert_array_equal(a, src)


@pytest.mark.gpu
@pytest.mark.parametrize("prog", ["RPCL", "PCRL", "CPRL"])
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_engine_off_grid_origin_equals_oracle(ci, prog):
    import grok_amd as G
    origin, prc, numres, tiles = CASES[ci]
    img = _img(ci, 37, 45)
    ref = O.encode(img, 8, **_okw(ci, prog))
    e = G.Engine(0)
    try:
        kw = dict(numresolution=numres, cblk=(4, 4), precincts=prc, prog_order=prog)
        if tiles:
            kw.update(tiles=tiles, tile_origin=(0, 0))
        cs = e.encode(img, 8, params=G.default_params(**kw), origin=origin)
        assert cs == ref
        np.testing.assert_array_equal(e.decode(ref), img)
    finally:
        e.close()
