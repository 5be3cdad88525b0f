"""Tiles coded with their own parameters: tile-part COD / COC / QCD / QCC (A.6; Grok's tile tcp,
CodeStreamDecompress read_cod / read_coc / read_qcd / read_qcc and Quantizer::read_SQcd_SQcc's
scoping).  Streams splice tiles of two oracle encodes (tests/tile_coding.py), so the answer is A's
decode with B's on the spliced tiles.  CPU: the oracle returns it, full, reduced and by the partial
(window) rule, and OpenJPEG 2.5.4 decodes the streams to the oracle's samples (9/7 tiles within 1:
OpenJPEG's own float path).  The engine half is tests/test_gpu_tile_coding.py."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
import openjpeg
from tile_coding import CASES, expected, stream

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def _irrev(name):
    H, W, ka, kb, tiles, form = CASES[name]
    return ka.get("irreversible") or kb.get("irreversible")


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_tile_coding(name):
    got, _ = O.decode(stream(name))
    np.testing.assert_array_equal(got, expected(name))


@pytest.mark.parametrize("name", ["levels_cblk", "coc_form", "prog_layers_sop"])
def test_oracle_tile_coding_tlm(name):
    got, _ = O.decode(stream(name, tlm=True))
    np.testing.assert_array_equal(got, expected(name))


@pytest.mark.parametrize("name", ["levels_cblk", "rev_to_irrev", "coc_form", "ht_tile", "ragged_tiles", "origin_tiles"])
def test_oracle_tile_coding_reduced(name):
    cs = stream(name)
    O.set_decode_reduce(1)
    try:
        got, _ = O.decode(cs)
    finally:
        O.set_decode_reduce(0)
    np.testing.assert_array_equal(got, expected(name, reduce=1))


def test_oracle_tile_coding_partial():
    got, _ = O.decode(stream("levels_cblk"), partial=True)
    np.testing.assert_array_equal(got, expected("levels_cblk", partial=True))


@pytest.mark.skipif(not openjpeg.available(), reason="libopenjp2 (Pillow's) not present")
@pytest.mark.parametrize("name", sorted(n for n in CASES if CASES[n][5] != "scope"))
def test_openjpeg_tile_coding(name):
    # (not the "scope" form: OpenJPEG's opj_j2k_read_qcd copies a tile QCD to every component in
    # marker order, over the tile's QCCs; Grok and A.6.5 let the QCC win, and the spliced data only
    # decodes that way: test_oracle_tile_coding)
    cs = stream(name)
    got, _ = O.decode(cs)
    for (dx, dy, r), g in zip(openjpeg.decode(cs), got):
        if _irrev(name):
            assert np.abs(r.astype(np.int64) - g).max() <= 1
        else:
            np.testing.assert_array_equal(r, g)


def test_tile_coding_reduce_past_a_tile_refused():
    # ragged_tiles' B tiles have two resolutions: reduce 2 leaves them none
    O.set_decode_reduce(2)
    try:
        with pytest.raises(RuntimeError, match="-7"):
            O.decode(stream("ragged_tiles"))
    finally:
        O.set_decode_reduce(0)


@pytest.mark.parametrize("name", sorted(CASES))
def test_engine_header_reads_tile_coding(name):
    # the engine's header reader (no GPU needed) takes the tile-part markers; a bad component
    # number in one is refused
    import grok_amd as G
    import j2k_markers as J
    cs = stream(name)
    info = G.probe_header(cs)
    H, W = CASES[name][:2]
    assert (info.w, info.h, info.numcomps) == (W, H, 3)
    with pytest.raises(ValueError, match="bad component number"):
        G.probe_header(J.insert_tile_part(cs, J.coc(cs, 3)))


@pytest.mark.parametrize("name", ["ht_and_part1", "mode_switches", "wide_block"])
def test_tile_cod_resets_main_coc(name):
    # a tile COD copies its SPcod to every component of the tile, over the main header's COCs
    # (read_cod :2603-2620; OpenJPEG's opj_j2k_read_cod likewise): the COC streams of
    # tests/test_coc.py with the main COD restated in the tile-part header decode their COC'd
    # components with component 0's coding, i.e. wrongly, and the same way in OpenJPEG 2.5.4
    import j2k_markers as J
    import test_coc
    cs = test_coc.stream(name)
    t = J.insert_tile_part(cs, J.cod(cs))
    got, _ = O.decode(t)
    want, _ = O.decode(cs)
    assert any(not np.array_equal(g, w) for g, w in zip(got, want))
    if openjpeg.available():
        for (dx, dy, r), g in zip(openjpeg.decode(t), got):
            np.testing.assert_array_equal(r, g)
