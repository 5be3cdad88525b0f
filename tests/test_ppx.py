"""Packed packet headers: PPM (main header) and PPT (tile-part headers), A.7.4 / A.7.5.

Grok's decoder reads them (CodeStreamDecompress read_ppm / read_ppt / merge_ppt, PPMMarker::merge;
T2Decompress.cpp:255-270 takes the packet headers from them, the bodies from the tile data); its
encoder writes neither.  Test streams come from the oracle's encoder with its packed-headers option
(the same packets, headers moved into PPT / PPM markers); OpenJPEG 2.5.4 decodes every one to the
source (lossless), which pins the streams and the oracle's reading of them.  GPU: the engine
decodes them to the oracle's samples, host and device streams, and windows."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
import openjpeg

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

CASES = {
    "plain": dict(numres=3),
    "tiles_sop_eph": dict(numres=4, tiles=(32, 32), sop=True, eph=True),
    "rpcl_layers_prc": dict(numres=3, nlayers=3, prog_order="RPCL", precincts=[(16, 16)]),
    "ht": dict(numres=3, cblk_sty=0x40),
    "modes_97": dict(numres=4, cblk_sty=0x05, irreversible=True),
}


def _img(name):
    rng = np.random.default_rng(sum(map(ord, name)))
    yy, xx = np.mgrid[0:70, 0:90]
    return np.stack([((xx * (c + 1) + yy * 2 + rng.integers(0, 32, size=(70, 90))) % 256) for c in range(3)]).astype(np.int32)


def stream(name, kind):
    return O.encode(_img(name), 8, packed_headers=kind, **CASES[name])


@pytest.mark.parametrize("kind", ["ppt", "ppm"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_packed_headers(name, kind):
    cs = stream(name, kind)
    marker = b"\xff\x61" if kind == "ppt" else b"\xff\x60"
    assert marker in cs
    got, _ = O.decode(cs)
    want, _ = O.decode(O.encode(_img(name), 8, **CASES[name]))   # the same packets, headers in place
    np.testing.assert_array_equal(got, want)
    if not CASES[name].get("irreversible"):
        np.testing.assert_array_equal(got, _img(name))


@pytest.mark.skipif(not openjpeg.available(), reason="libopenjp2 (Pillow's) not present")
@pytest.mark.parametrize("kind", ["ppt", "ppm"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_openjpeg_packed_headers(name, kind):
    cs = stream(name, kind)
    ref = openjpeg.decode(cs)
    got, _ = O.decode(cs)
    for (dx, dy, r), g in zip(ref, got):
        if CASES[name].get("irreversible"):
            assert np.abs(r.astype(np.int64) - g).max() <= 1   # (9/7: OpenJPEG's own float path)
        else:
            np.testing.assert_array_equal(r, g)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["ppt", "ppm"])
@pytest.mark.parametrize("name", sorted(CASES))
def test_engine_packed_headers(name, kind):
    import grok_amd as G
    import torch
    cs = stream(name, kind)
    want, _ = O.decode(cs)
    e = G.Engine(0)
    try:
        np.testing.assert_array_equal(e.decode(cs), want)
        d = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
        np.testing.assert_array_equal(e.decode(d, len(cs)), want)
        part, _ = O.decode(cs, partial=True)
        np.testing.assert_array_equal(e.decode_window(cs, (5, 7, 61, 50)), part[:, 7:50, 5:61])
    finally:
        e.close()
