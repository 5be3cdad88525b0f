"""Progression orders LRCP / RLCP / RPCL / PCRL / CPRL (COD SGcod byte, grk_compress -p;
PacketIter.cpp:100-335) on the HIP path vs the oracle.

The engine orders a tile's packets by sorting precincts on their first sample in the
reference grid (gk_engine.cpp packet_order); the oracle walks Grok's position iterator
literally (y += dy - y % dy, generatePrecinctIndex).  Bar: encode byte-identical (single
layer, precincts, tiles + PLT, PCRD layers), decode sample-identical, window decodes
(PLT packet skipping in these orders) equal to crops.  Parity with Grok unpinned: no
reference-held fixture uses a progression other than LRCP.
"""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu

PROGS = ["RLCP", "RPCL", "PCRL", "CPRL"]


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


def _img(seed, c, h, w, bits=8):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = (np.sin(xx / 13.0 + seed) * np.cos(yy / 9.0) + 1) * (1 << (bits - 2))
    return np.clip(base[None].repeat(c, 0) + rng.integers(0, 1 << (bits - 3), size=(c, h, w)), 0,
                   (1 << bits) - 1).astype(np.int32)


CASES = [
    dict(numres=4, cblk=(16, 16)),
    dict(numres=5, cblk=(32, 32), precincts=[(64, 64), (32, 32)]),
    dict(numres=4, cblk=(16, 16), precincts=[(32, 32)], tiles=(64, 96), plt=True, tlm=True),
    dict(numres=4, cblk=(32, 32), precincts=[(64, 64)], layer_rate=[30, 10, 3]),
    dict(numres=3, cblk=(16, 16), precincts=[(32, 32)], irreversible=True, layer_rate=[40, 20]),
]


def _gk(k, prog):
    import grok_amd as G
    kw = dict(numresolution=k["numres"], cblk=k["cblk"], prog_order=prog)
    for n in ("precincts", "tiles", "plt", "tlm", "irreversible", "layer_rate"):
        if n in k:
            kw[n] = k[n]
    return G.default_params(**kw)


def _ok(k, prog):
    kw = dict(numres=k["numres"], cblk=k["cblk"], prog_order=prog)
    for n in ("precincts", "tiles", "plt", "tlm", "irreversible", "layer_rate"):
        if n in k:
            kw[n] = k[n]
    return kw


@pytest.mark.parametrize("prog", PROGS)
@pytest.mark.parametrize("ci", range(len(CASES)))
def test_progression_vs_oracle(eng, prog, ci):
    k = CASES[ci]
    img = _img(ci, 3, 150, 170)
    cs = eng.encode(img, 8, params=_gk(k, prog))
    ref = O.encode(img, 8, **_ok(k, prog))
    assert cs == ref
    dec = eng.decode(ref)
    np.testing.assert_array_equal(dec, O.decode(ref)[0])
    if "layer_rate" not in k and not k.get("irreversible"):
        np.testing.assert_array_equal(dec, img)


@pytest.mark.parametrize("prog", ["RPCL", "PCRL", "CPRL"])
def test_progression_window_decode(eng, prog):
    k = CASES[2]
    img = _img(7, 3, 150, 170)
    cs = eng.encode(img, 8, params=_gk(k, prog))
    for (x0, y0, x1, y1) in [(0, 0, 40, 30), (70, 60, 150, 140), (100, 5, 170, 150)]:
        win = eng.decode_window(cs, (x0, y0, x1, y1))
        np.testing.assert_array_equal(win, img[:, y0:y1, x0:x1])


@pytest.mark.parametrize("prog", ["LRCP", "RPCL"])
@pytest.mark.parametrize("plt", [False, True])
def test_layer_limited_decode(eng, prog, plt):
    """grk_decompress -l (cp_layer): the first n layers only, vs the oracle's same limit;
    quality grows with n and n = all equals the full decode."""
    k = dict(numres=4, cblk=(32, 32), precincts=[(64, 64)], layer_rate=[40, 10, 2], plt=plt)
    img = _img(11, 3, 150, 170)
    cs = eng.encode(img, 8, params=_gk(k, prog))
    full = eng.decode(cs)
    errs = []
    try:
        for n in (1, 2, 3):
            eng.set_decode_layers(n)
            O.set_decode_layers(n)
            dec = eng.decode(cs)
            np.testing.assert_array_equal(dec, O.decode(cs)[0])
            errs.append(np.abs(dec.astype(np.int64) - img).mean())
    finally:
        eng.set_decode_layers(0)
        O.set_decode_layers(0)
    np.testing.assert_array_equal(dec, full)
    assert errs[0] > errs[1] > errs[2]


POCS = [
    [(0, 0, 1, 3, 3, "RLCP"), (0, 0, 3, 4, 3, "LRCP")],
    [(0, 0, 2, 4, 2, "CPRL"), (0, 2, 2, 4, 3, "RPCL"), (0, 0, 3, 4, 3, "PCRL")],
    [(1, 0, 3, 4, 3, "RPCL"), (0, 0, 3, 1, 3, "LRCP")],
]


@pytest.mark.parametrize("pi", range(len(POCS)))
def test_progression_order_changes(eng, pi):
    """POC (A.6.6; PacketIter over the tile's progressions, update_include) as Grok writes it:
    tile 0's list in the main header and in each tile's first tile part, one tile part per
    entry (CodeStreamCompress.cpp:839-840, 870-875, 902-946), packets entry by entry, each once
    (overlapping entries: the later ones' parts skip what was written), the rate control's
    simulation in the tile's own progression.  Encode byte-identical to the oracle, decodes
    equal (whole, window)."""
    import grok_amd as G
    img = _img(20 + pi, 3, 150, 170)
    for kw in (dict(tiles=(64, 96), plt=True, tlm=True), dict(precincts=[(32, 32)], layer_rate=[20, 5, 0])):
        gkw = dict(kw)
        if "layer_rate" in gkw:
            gkw["numlayers"] = len(gkw["layer_rate"])
        cs = eng.encode(img, 8, params=G.default_params(numresolution=4, cblk=(16, 16), pocs=POCS[pi], **gkw))
        ref = O.encode(img, 8, numres=4, cblk=(16, 16), pocs=POCS[pi], **kw)
        assert cs == ref
        np.testing.assert_array_equal(eng.decode(cs), img)
        if "tiles" in kw:
            np.testing.assert_array_equal(eng.decode_window(cs, (30, 20, 160, 120)), img[:, 20:120, 30:160])


def test_incomplete_poc_refused(eng):
    """CodeStreamCompress::validateProgressionOrders (CodeStreamCompress.cpp:1685-1747): POC
    entries that leave a (layer, resolution, component) packet uncovered are refused ("POC:
    missing packets") instead of silently dropping the packet's code-blocks."""
    import grok_amd as G
    img = _img(30, 3, 64, 80)
    for pocs in ([(0, 0, 1, 4, 3, "LRCP")],                              # layers 1.. of 2 missing
                 [(0, 0, 2, 3, 3, "RLCP")],                              # resolution 3 missing
                 [(0, 0, 2, 4, 2, "CPRL"), (1, 2, 2, 4, 3, "RPCL")]):    # (r 0, c 2) missing
        p = G.default_params(numresolution=4, cblk=(16, 16), layer_rate=[20, 0], pocs=pocs)
        with pytest.raises(RuntimeError, match="POC: missing packets"):
            eng.encode(img, 8, params=p)
    # the engine stays usable and a covering list still encodes
    p = G.default_params(numresolution=4, cblk=(16, 16), layer_rate=[20, 0], pocs=[(0, 0, 2, 4, 3, "RLCP")])
    assert eng.encode(img, 8, params=p) == O.encode(img, 8, numres=4, cblk=(16, 16), layer_rate=[20, 0],
                                                    pocs=[(0, 0, 2, 4, 3, "RLCP")])
