"""Subsampled components (SIZ XRsiz / YRsiz) in the oracle, pinned by OpenJPEG 2.5.4.

The oracle restates Grok's subsampling rules (tests/subsampling_cases.py lists them); OpenJPEG,
driven through its C API (tests/openjpeg.py), decodes every oracle-encoded case to the oracle's own
decode, component by component at each component's size, and the 5/3 cases round-trip losslessly.
The C-ABI's header probe (no GPU) reports the subsampling.  The engine half is
tests/test_gpu_subsampling.py."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
import openjpeg
from subsampling_cases import CASES, comp_shape, oracle_kw, planes

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def _encode(name):
    W, H, sub, prec, kw = CASES[name]
    return O.encode(planes(name), prec, size=(W, H), **oracle_kw(name))


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_subsampled_round_trip(name):
    W, H, sub, prec, kw = CASES[name]
    cs = _encode(name)
    got, p = O.decode(cs)
    assert p == prec
    origin = kw.get("origin") or kw.get("tile_origin") or (0, 0)
    assert [g.shape for g in got] == [comp_shape(W, H, dx, dy, origin) for dx, dy in sub]
    if not kw.get("irreversible") and not kw.get("layer_rate"):
        for g, src in zip(got, planes(name)):
            np.testing.assert_array_equal(g, src)


@pytest.mark.skipif(not openjpeg.available(), reason="libopenjp2 (Pillow's) not present")
@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_subsampled_equals_openjpeg(name):
    W, H, sub, prec, kw = CASES[name]
    cs = _encode(name)
    got, _ = O.decode(cs)
    ref = openjpeg.decode(cs)
    assert [(r[0], r[1]) for r in ref] == [tuple(d) for d in sub]
    for (dx, dy, r), g in zip(ref, got):
        np.testing.assert_array_equal(r, g)


def test_oracle_subsampled_reduce_shapes():
    # reduced decode: each component's rectangle on its grid, both edges ceil(x / 2^r)
    name = "offset_odd"
    W, H, sub, prec, kw = CASES[name]
    cs = _encode(name)
    O.set_decode_reduce(1)
    try:
        got, _ = O.decode(cs)
    finally:
        O.set_decode_reduce(0)
    x0, y0 = kw["origin"]
    for (dx, dy), g in zip(sub, got):
        cx0, cy0, cx1, cy1 = -(-x0 // dx), -(-y0 // dy), -(-(x0 + W) // dx), -(-(y0 + H) // dy)
        assert g.shape == (-(-cy1 // 2) - -(-cy0 // 2), -(-cx1 // 2) - -(-cx0 // 2))


def test_oracle_no_mct_across_grids():
    # the first three components on different grids: Grok clears the MCT flag (COD SGcod byte 4)
    cs = _encode("420_53")
    cod = cs.index(b"\xff\x52")
    assert cs[cod + 4 + 4] == 0
    cs2 = _encode("mixed4")   # (1,1), (1,1), (2,2): still different
    cod2 = cs2.index(b"\xff\x52")
    assert cs2[cod2 + 4 + 4] == 0


def test_capi_probe_components():
    import grok_amd as G
    for name in ("420_53", "cprl_dx3", "mono12_sub"):
        W, H, sub, prec, kw = CASES[name]
        cs = _encode(name)
        assert G.probe_components(cs) == [tuple(d) for d in sub]
        info = G.probe_header(cs)
        assert (info.w, info.h, info.numcomps) == (W, H, len(sub))
