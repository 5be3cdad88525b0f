"""COC / QCC and tile-part COD / QCD markers in the oracle decoder.

Grok reads COC / QCC (CodeStreamDecompress read_coc / read_qcc) and tile-part COD / COC / QCD / QCC
as per-component / per-tile overrides of the main COD / QCD.  A main-header QCC / COC is applied
to its component (tests/test_qcc.py, tests/test_coc.py); tile-part markers set the tile's own coding
(tests/test_tile_coding.py for streams coded that way).  Here the committed Grok fixtures get
markers spliced in (tests/j2k_markers.py): markers that restate the main header decode exactly as
the stream without them (some encoders write them unconditionally); markers that change the first
tile's code-block style, guard bits or ROI shift decode as OpenJPEG 2.5.4 decodes them (sample for sample,
9/7 included); a tile COD with one more layer than the tile holds reads the tile as truncated, i.e.
as before.  The engine half is tests/test_gpu_override_markers.py.
"""
import os
import sys

import numpy as np
import pytest

from conftest import FIXTURES, ROOT
import j2k_markers as J
import openjpeg

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

NAMES = ["rgb8_tiles_xl", "rgb12_97_r", "mono16_ht_tiles", "rgb8_prc"]


def _fx(name):
    return next(f for f in FIXTURES if f.name == name)


def restating(cs):
    n = J.ncomp(cs)
    segs = b"".join(J.coc(cs, c) + J.qcc(cs, c) for c in range(n))
    return J.insert_tile_part(J.insert_main(cs, segs), J.cod(cs) + J.qcd(cs) + J.coc(cs, n - 1) + J.qcc(cs, 0))


def changing(cs):
    # (a main-header COC that changes its component's coding is applied: tests/test_coc.py)
    yield "tile COD", J.insert_tile_part(cs, J.cod(cs, layers_add=1))
    yield "tile COC", J.insert_tile_part(cs, J.coc(cs, 0, sty_xor=0x08))
    yield "tile QCC", J.insert_tile_part(cs, J.qcc(cs, 0, guard_add=1))
    yield "tile RGN", J.insert_tile_part(cs, J.rgn(cs, 0, 3))


def refused(cs):
    yield "COC bad component", J.insert_main(cs, J.coc(cs, J.ncomp(cs)))
    yield "tile COC bad component", J.insert_tile_part(cs, J.coc(cs, J.ncomp(cs)))


@pytest.mark.parametrize("name", NAMES)
def test_restating_markers_decode_as_without(name):
    fx = _fx(name)
    want, prec = O.decode(fx.cs)
    got, prec2 = O.decode(restating(fx.cs))
    assert prec == prec2
    np.testing.assert_array_equal(got, want)
    np.testing.assert_array_equal(got, fx.grok_decoded)


@pytest.mark.parametrize("name", NAMES)
def test_changing_tile_markers_applied(name):
    fx = _fx(name)
    for what, cs in changing(fx.cs):
        if what == "tile COD":   # (the extra layer's packets are absent: a truncated tile)
            np.testing.assert_array_equal(O.decode(cs)[0], fx.grok_decoded)
        elif fx.ht and what == "tile COC":   # HT with a Part-1 mode switch (CodeStreamDecompress.cpp:1781)
            with pytest.raises(RuntimeError, match="failed: -2"):
                O.decode(cs)
        elif what == "tile RGN":
            # maxshift ROI over data coded without one: every nonzero index is at or above the
            # shift once the bit-planes move up, so the descale restores it (OpenJPEG agrees);
            # the tile's shift is read, the samples stay.  (HT: OpenJPEG refuses; the engine
            # half compares with the oracle.)
            got, _ = O.decode(cs)
            if fx.ht:
                continue
            np.testing.assert_array_equal(got, fx.grok_decoded)
            if openjpeg.available():
                for (dx, dy, r), g in zip(openjpeg.decode(cs), got):
                    np.testing.assert_array_equal(r, g)
        elif fx.ht:   # HT places magnitudes by the zero bit-plane count alone: guard bits do not move them
            np.testing.assert_array_equal(O.decode(cs)[0], fx.grok_decoded)
        else:
            got, _ = O.decode(cs)
            assert not np.array_equal(got, fx.grok_decoded), what
            if openjpeg.available():
                for (dx, dy, r), g in zip(openjpeg.decode(cs), got):
                    np.testing.assert_array_equal(r, g, err_msg=what)


@pytest.mark.parametrize("name", NAMES)
def test_bad_component_refused(name):
    fx = _fx(name)
    for what, cs in refused(fx.cs):
        with pytest.raises(RuntimeError, match="failed: -2"):
            O.decode(cs)


@pytest.mark.parametrize("name", NAMES)
def test_main_qcc_applies_to_its_component(name):
    # a main-header QCC with one more guard bit raises that component's band bit-plane counts
    # (Quantizer.cpp:47), so a Part-1 block's bit-planes (band count less the packet header's zero
    # bit-planes) move up one: the stream decodes, differently; HT places the magnitude by the
    # zero bit-plane count alone (k_msbs), so its samples stay
    fx = _fx(name)
    n = J.ncomp(fx.cs)
    got, _ = O.decode(J.insert_main(fx.cs, J.qcc(fx.cs, n - 1, guard_add=1)))
    assert got.shape == fx.grok_decoded.shape
    if fx.ht:
        np.testing.assert_array_equal(got, fx.grok_decoded)
    else:
        assert not np.array_equal(got, fx.grok_decoded)


@pytest.mark.parametrize("marker", [0xFF74, 0xFF75, 0xFF77, 0xFF78, 0xFF79])
def test_part2_markers_refused(marker):
    # Part-2 extensions (MCT / MCC / MCO / CBD / ATK) change the decode; refused rather than ignored
    fx = _fx("rgb8_tiles_xl")
    cs = J.insert_main(fx.cs, bytes([marker >> 8, marker & 0xFF, 0, 4, 0, 0]))
    with pytest.raises(RuntimeError, match="failed: -2"):
        O.decode(cs)
    import grok_amd as G
    with pytest.raises(ValueError, match="Part-2"):
        G.probe_header(cs)


def test_part2_array_mct_refused():
    fx = _fx("rgb8_tiles_xl")
    cs = bytearray(fx.cs)
    cod = cs.index(b"\xff\x52")
    cs[cod + 4 + 4] = 2   # SGcod MCT = 2: a Part-2 array transform
    with pytest.raises(RuntimeError, match="failed: -2"):
        O.decode(bytes(cs))
    import grok_amd as G
    with pytest.raises(ValueError, match="Part-2"):
        G.probe_header(bytes(cs))
