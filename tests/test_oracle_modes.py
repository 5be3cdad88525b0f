"""Oracle self-consistency for the code-block mode switches (CPU): every combination of
the reference's non-regression list round-trips losslessly through the oracle's encoder
and segment-aware decoder, with one and several quality layers.  (Parity with Grok for
these modes is unpinned: no reference-held fixture carries such a codestream.)"""
import numpy as np
import pytest

import oracle as O


@pytest.mark.parametrize("sty", [1, 2, 4, 8, 16, 32, 5, 17, 20, 38, 63])
@pytest.mark.parametrize("layers", [None, [10, 0]])
def test_oracle_modes_roundtrip(sty, layers):
    rng = np.random.default_rng(sty)
    img = rng.integers(0, 4096, size=(1, 70, 90)).astype(np.int32)
    img = (img // 8 + np.arange(90)[None, None, :] * 40) % 4096
    cs = O.encode(img.astype(np.int32), 12, numres=3, cblk=(32, 32), cblk_sty=sty, layer_rate=layers)
    np.testing.assert_array_equal(O.decode(cs)[0], img)


def test_oracle_modes_change_stream():
    rng = np.random.default_rng(0)
    img = rng.integers(0, 256, size=(1, 64, 64)).astype(np.int32)
    base = O.encode(img, 8, numres=3, cblk=(32, 32))
    for sty in (1, 2, 4, 8, 16, 32):
        assert O.encode(img, 8, numres=3, cblk=(32, 32), cblk_sty=sty) != base


@pytest.mark.parametrize("bits,c", [(8, 3), (12, 1), (16, 1)])
def test_oracle_ht97_roundtrip(bits, c):
    """HT + 9/7 (standard-correct in place of R-BUG-2): decodes close to the source."""
    rng = np.random.default_rng(bits)
    yy, xx = np.mgrid[0:90, 0:110]
    base = (np.sin(xx / 9.0) * np.cos(yy / 7.0) + 1) * (1 << (bits - 2))
    img = np.clip(base[None].repeat(c, 0) + rng.integers(0, 1 << (bits - 4), size=(c, 90, 110)), 0,
                  (1 << bits) - 1).astype(np.int32)
    cs = O.encode(img, bits, numres=5, cblk_sty=0x40, irreversible=True)
    dec = O.decode(cs)[0]
    mse = np.mean((dec.astype(np.float64) - img) ** 2)
    assert 10 * np.log10(((1 << bits) - 1) ** 2 / max(mse, 1e-12)) >= 45.0


@pytest.mark.parametrize("prog", ["LRCP", "RLCP", "RPCL", "PCRL", "CPRL"])
def test_oracle_progressions_roundtrip(prog):
    """Every progression order round-trips (precincts, tiles) and changes the packet order."""
    rng = np.random.default_rng(5)
    img = rng.integers(0, 256, size=(3, 100, 120)).astype(np.int32)
    kw = dict(numres=4, cblk=(16, 16), precincts=[(32, 32)], tiles=(64, 64))
    cs = O.encode(img, 8, prog_order=prog, **kw)
    np.testing.assert_array_equal(O.decode(cs)[0], img)
    if prog != "LRCP":
        assert cs != O.encode(img, 8, **kw)


def test_oracle_layer_limit():
    rng = np.random.default_rng(6)
    img = (rng.integers(0, 64, size=(1, 96, 96)) + np.arange(96)[None, None, :]).astype(np.int32)
    cs = O.encode(img, 8, numres=3, cblk=(32, 32), layer_rate=[30, 8, 0])
    errs = []
    try:
        for n in (1, 2, 3):
            O.set_decode_layers(n)
            errs.append(np.abs(O.decode(cs)[0].astype(np.int64) - img).mean())
    finally:
        O.set_decode_layers(0)
    assert errs[0] > errs[1] > errs[2] == 0


@pytest.mark.parametrize("prog,div", [("LRCP", "L"), ("LRCP", "R"), ("RPCL", "R"), ("CPRL", "C")])
def test_oracle_tile_part_generation(prog, div):
    rng = np.random.default_rng(7)
    img = rng.integers(0, 256, size=(3, 90, 100)).astype(np.int32)
    cs = O.encode(img, 8, numres=3, cblk=(16, 16), prog_order=prog, tile_parts=div, tiles=(64, 64), tlm=True, plt=True,
                  layer_rate=[10, 0])
    assert cs.count(b"\xff\x90") > 4   # several SOT markers per tile
    np.testing.assert_array_equal(O.decode(cs)[0], img)
