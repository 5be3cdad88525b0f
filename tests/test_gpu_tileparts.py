"""Tiles split over several tile parts (SOT TPsot / TNsot, ISO 15444-1 A.4.2): the decoder
continues a tile's packet sequence across its tile parts (T2Decompress over the parts in
order; gk_engine.cpp merge_tile_parts).  Streams are made by re-cutting single-part
streams at packet boundaries (PLT gives them), which leaves the coded data unchanged, so
the bar is: the split stream decodes sample-identical to the original, whole and by
window, with and without PLT in the parts.  Grok reads such streams (its own encoder
writes them with -u); no reference-held fixture has one.
"""
import struct

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


def _img(seed, c, h, w):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = (np.sin(xx / 10.0 + seed) * np.cos(yy / 8.0) + 1) * 64
    return np.clip(base[None].repeat(c, 0) + rng.integers(0, 32, size=(c, h, w)), 0, 255).astype(np.int32)


def _plt_lengths(body):
    out, v = [], 0
    for b in body:
        v = (v << 7) | (b & 0x7F)
        if not b & 0x80:
            out.append(v)
            v = 0
    return out


def _plt_marker(lens):
    v = bytearray()
    for n in lens:
        groups = []
        while True:
            groups.append(n & 0x7F)
            n >>= 7
            if not n:
                break
        for i, g in enumerate(reversed(groups)):
            v.append(g | (0x80 if i < len(groups) - 1 else 0))
    return b"\xff\x58" + struct.pack(">H", 3 + len(v)) + b"\x00" + bytes(v)


def split_tile_parts(cs, nparts, keep_plt):
    """Re-cut every tile of a PLT-carrying codestream into up to `nparts` tile parts."""
    cs = bytes(cs)
    pos = cs.index(b"\xff\x90")
    out = bytearray(cs[:pos])
    while cs[pos:pos + 2] == b"\xff\x90":
        isot, psot = struct.unpack(">HI", cs[pos + 4:pos + 10])
        end = pos + psot
        j, lens = pos + 12, []
        while cs[j:j + 2] != b"\xff\x93":
            m, L = struct.unpack(">HH", cs[j:j + 4])
            if m == 0xFF58:
                lens += _plt_lengths(cs[j + 5:j + 2 + L])
            j += 2 + L
        data = j + 2
        assert sum(lens) == end - data
        k = min(nparts, len(lens))
        cuts = [round(i * len(lens) / k) for i in range(k + 1)]
        p = data
        for t in range(k):
            pl = lens[cuts[t]:cuts[t + 1]]
            body = cs[p:p + sum(pl)]
            p += sum(pl)
            hdr = _plt_marker(pl) if keep_plt else b""
            psot_t = 12 + len(hdr) + 2 + len(body)
            out += b"\xff\x90" + struct.pack(">HHIBB", 10, isot, psot_t, t, k) + hdr + b"\xff\x93" + body
        pos = end
    out += cs[pos:]
    return bytes(out)


@pytest.mark.parametrize("prog", ["LRCP", "RPCL", "CPRL"])
@pytest.mark.parametrize("keep_plt", [False, True])
def test_split_tile_parts_decode(eng, prog, keep_plt):
    import grok_amd as G
    img = _img(3, 3, 160, 190)
    p = G.default_params(numresolution=4, cblk=(16, 16), precincts=[(32, 32)], tiles=(64, 96), plt=True,
                         prog_order=prog, layer_rate=[30, 8, 0], numlayers=3)
    cs = eng.encode(img, 8, params=p)
    full = eng.decode(cs)
    for n in (2, 3, 7):
        sp = split_tile_parts(cs, n, keep_plt)
        assert sp != cs
        np.testing.assert_array_equal(eng.decode(sp), full)
        win = (50, 40, 170, 150)
        np.testing.assert_array_equal(eng.decode_window(sp, win), full[:, 40:150, 50:170])


def test_split_tile_parts_device_stream(eng):
    import torch
    import grok_amd as G
    img = _img(4, 1, 130, 140)
    cs = eng.encode(img, 8, params=G.default_params(numresolution=3, cblk=(32, 32), tiles=(64, 64), plt=True))
    sp = split_tile_parts(cs, 3, True)
    dev = torch.frombuffer(bytearray(sp), dtype=torch.uint8).cuda()
    np.testing.assert_array_equal(eng.decode(dev, length=len(sp)), img)


GEN = [("LRCP", "L"), ("LRCP", "R"), ("RLCP", "R"), ("RPCL", "R"), ("CPRL", "C"), ("LRCP", "C")]


@pytest.mark.parametrize("prog,div", GEN)
def test_tile_part_generation_vs_oracle(eng, prog, div):
    """grk_compress -u L|R|C (enableTilePartGeneration): a new tile part whenever the
    progression's index up to the divider changes (getNumTilePartsForProgression), PLT in
    the first part, TLM with one entry per part, 14 bytes per extra part off the rate
    budget (updateRates).  Encode byte-identical to the oracle; decodes equal."""
    import oracle as O
    import grok_amd as G
    img = _img(8, 3, 150, 170)
    for kw in (dict(tiles=(64, 96), tlm=True, plt=True), dict(layer_rate=[30, 8, 2], precincts=[(64, 64)])):
        gkw = dict(kw)
        if "layer_rate" in gkw:
            gkw["numlayers"] = len(gkw["layer_rate"])
        cs = eng.encode(img, 8, params=G.default_params(numresolution=4, cblk=(16, 16), prog_order=prog,
                                                        tile_parts=div, **gkw))
        ref = O.encode(img, 8, numres=4, cblk=(16, 16), prog_order=prog, tile_parts=div, **kw)
        assert cs == ref
        np.testing.assert_array_equal(eng.decode(cs), O.decode(ref)[0])
        if "tiles" in kw:
            np.testing.assert_array_equal(eng.decode_window(cs, (20, 30, 150, 140)), img[:, 30:140, 20:150])


def test_tile_part_divider_behind_position_refused(eng):
    import grok_amd as G
    img = _img(9, 1, 64, 64)
    with pytest.raises(Exception):
        eng.encode(img, 8, params=G.default_params(numresolution=3, prog_order="PCRL", tile_parts="C"))
