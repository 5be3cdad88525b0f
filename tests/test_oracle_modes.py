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


# ------------------------------------------------------------------ SOP / EPH and fixed quality
# grk_compress -S / -E (csty SOP / EPH bits, T2Compress.cpp:286-320 writer, T2Decompress.cpp:
# 226-250 / 469-486 reader) and -q PSNR layers (allocationByQuality, TileProcessor.cpp:1296-1322).
# No Grok fixture holds these streams (parity unpinned against Grok itself: the oracle
# restates the writer / reader / bisection); the GPU suite holds the HIP path equal to the oracle.
from grok_amd.synth import synth_image as _synth  # noqa: E402


def _sop_eph_positions(cs):
    i, out = cs.find(b"\xff\x90"), []
    while True:
        j = cs.find(b"\xff\x91", i)
        if j < 0:
            return out
        out.append(j)
        i = j + 2


@pytest.mark.parametrize("kw", [dict(sop=True), dict(eph=True), dict(sop=True, eph=True),
                                dict(sop=True, eph=True, layer_rate=[20.0, 5.0]),
                                dict(sop=True, eph=True, tiles=(128, 128), plt=True, tlm=True, layer_rate=[10.0]),
                                dict(sop=True, eph=True, prog_order="RPCL", precincts=[(64, 64)]),
                                dict(sop=True, eph=True, tile_parts="R", tiles=(128, 128))],
                         ids=["sop", "eph", "sop_eph", "sop_eph_r", "sop_eph_tiles_plt", "sop_eph_rpcl_prc", "sop_eph_tp"])
def test_sop_eph_round_trip(kw):
    img = _synth(200, 300, 3, 8, 5).astype(np.int32)
    cs = O.encode(img, 8, **kw)
    dec, _ = O.decode(cs)
    if "layer_rate" not in kw:
        np.testing.assert_array_equal(dec, img)
    # Scod carries the bits; SOP segments count the packets of their tile from 0
    cod = cs.find(b"\xff\x52")
    scod = cs[cod + 4]
    assert bool(scod & 2) == bool(kw.get("sop")) and bool(scod & 4) == bool(kw.get("eph"))
    if kw.get("sop"):
        pos = _sop_eph_positions(cs)
        assert pos and all(cs[p + 2:p + 4] == b"\x00\x04" for p in pos)
        first = int.from_bytes(cs[pos[0] + 4:pos[0] + 6], "big")
        assert first == 0
    plain = O.encode(img, 8, **{k: v for k, v in kw.items() if k not in ("sop", "eph")})
    if "layer_rate" not in kw:   # lossless: the same packets plus 6 / 2 bytes each
        npk = cs.count(b"\xff\x91") if kw.get("sop") else cs.count(b"\xff\x92")
        extra = npk * ((6 if kw.get("sop") else 0) + (2 if kw.get("eph") else 0))
        plt_extra = 0
        assert len(cs) - len(plain) >= extra + plt_extra


def test_sop_counter_mismatch_is_refused():
    img = _synth(64, 64, 1, 8, 3).astype(np.int32)
    cs = bytearray(O.encode(img, 8, sop=True))
    p = _sop_eph_positions(bytes(cs))[1]
    cs[p + 5] ^= 1
    with pytest.raises(RuntimeError):
        O.decode(bytes(cs))


@pytest.mark.parametrize("kw", [dict(quality=[30.0, 40.0]), dict(quality=[28.0, 36.0, 0.0]),
                                dict(quality=[35.0], irreversible=True), dict(quality=[30.0, 38.0], tiles=(128, 128))],
                         ids=["q30_40", "q28_36_lossless", "q35_97", "q30_38_tiles"])
def test_fixed_quality_layers(kw):
    img = _synth(200, 300, 3, 8, 5).astype(np.int32)
    cs = O.encode(img, 8, **kw)
    dec, _ = O.decode(cs)
    q = kw["quality"]
    if q[-1] == 0:
        np.testing.assert_array_equal(dec, img)
    else:   # the targets are met approximately (the distortion estimates are Grok's)
        mse = float(((dec.astype(np.float64) - img) ** 2).mean())
        assert 10 * np.log10(255.0 ** 2 / mse) > q[-1] - 3.0
    # more layers decoded -> more quality
    O.set_decode_layers(1)
    try:
        d1, _ = O.decode(cs)
    finally:
        O.set_decode_layers(0)
    assert np.abs(d1.astype(np.int64) - img).sum() >= np.abs(dec.astype(np.int64) - img).sum()
