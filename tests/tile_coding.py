"""Codestreams whose tiles are coded with different parameters (tile-part COD / COC / QCD / QCC,
ISO 15444-1 A.6.1 / A.6.2 / A.6.4 / A.6.5), made by splicing tiles of two oracle encodes.

Neither Grok's encoder nor the oracle's writes tile-part coding markers (grk_cparameters has one
coding style per image), so test streams are assembled: the image is encoded twice, with the base
parameters A and the tile parameters B (the same tile grid, one tile part per tile); the parts of
the chosen tiles are taken from B's stream and given tile-part markers that state B's coding, the
other parts stay A's.  A tile's packets depend only on its own samples and coding, so a decoder must
return B's decode on those tiles and A's elsewhere; OpenJPEG 2.5.4 does (tests/test_tile_coding.py).

Marker forms for a B tile:
  "cod":   COD(B) + QCD(B)                 (read_cod copies SPcod to every component)
  "coc":   COC(c, B) + QCC(c, B) for every c (B's Scod / SGcod must equal A's)
  "scope": QCC(c, B) for every c, COD(B), then QCD(A): a tile QCC wins over the tile QCD in any
           order (Quantizer.cpp:208-235), so A's QCD is ignored
  "rgn":   B's RGN markers (B = A with an ROI shift: the tile's own ROI, read_rgn)
"""
import os
import struct
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def _main(cs):
    """({code: body} of the first of each main-header marker, [raw segments], first SOT offset)."""
    i, first, segs = 2, {}, []
    while True:
        m, L = struct.unpack(">HH", cs[i:i + 4])
        if m == 0xFF90:
            return first, segs, i
        first.setdefault(m, cs[i + 4:i + 2 + L])
        segs.append((m, cs[i:i + 2 + L]))
        i += 2 + L


def _parts(cs, sot):
    """{tile: (tile-part header segments after SOT, data after SOD)}; one part per tile."""
    out, i = {}, sot
    while i + 12 <= len(cs) and cs[i:i + 2] == b"\xff\x90":
        isot, psot, tpsot, tnsot = struct.unpack(">HIBB", cs[i + 4:i + 12])
        assert tpsot == 0 and tnsot in (0, 1) and psot
        j = i + 12
        while cs[j:j + 2] != b"\xff\x93":
            j += 2 + struct.unpack(">H", cs[j + 2:j + 4])[0]
        out[isot] = (cs[i + 12:j], cs[j + 2:i + psot])
        i += psot
    return out


def _seg(code, payload):
    return struct.pack(">HH", code, 2 + len(payload)) + payload


def _coc_form(cod):
    return bytes([cod[0] & 1]) + bytes(cod[5:])


def marker_segments(a_main, b_main, nc, form, b_segs=()):
    cod_b, qcd_b, qcd_a = b_main[0xFF52], b_main[0xFF5C], a_main[0xFF5C]
    cw = 1 if nc <= 256 else 2
    cid = lambda c: c.to_bytes(cw, "big")
    if form == "cod":
        return _seg(0xFF52, cod_b) + _seg(0xFF5C, qcd_b)
    if form == "coc":
        cod_a = a_main[0xFF52]
        assert cod_a[0] & 6 == cod_b[0] & 6 and cod_a[1:5] == cod_b[1:5], "COC form needs B's SOP / EPH and SGcod as A's"
        return b"".join(_seg(0xFF53, cid(c) + _coc_form(cod_b)) + _seg(0xFF5D, cid(c) + qcd_b) for c in range(nc))
    if form == "scope":
        return (b"".join(_seg(0xFF5D, cid(c) + qcd_b) for c in range(nc)) + _seg(0xFF52, cod_b) +
                _seg(0xFF5C, qcd_a))
    if form == "rgn":
        return b"".join(seg for m, seg in b_segs if m == 0xFF5E)
    raise ValueError(form)


def splice(cs_a, cs_b, tiles, form="cod", tlm=False):
    """cs_a with the parts of `tiles` taken from cs_b, each behind the tile-part markers of `form`
    stating B's coding.  tlm: write a TLM marker (Ttlm 16 bits, Ptlm 32 bits) for the result."""
    a_main, a_segs, a_sot = _main(cs_a)
    b_main, b_segs, b_sot = _main(cs_b)
    nc = struct.unpack(">H", a_main[0xFF51][34:36])[0]
    pa, pb = _parts(cs_a, a_sot), _parts(cs_b, b_sot)
    assert sorted(pa) == sorted(pb)
    body, lens = b"", []
    for t in sorted(pa):
        hdr, data = pb[t] if t in tiles else pa[t]
        if t in tiles:
            hdr = marker_segments(a_main, b_main, nc, form, b_segs) + hdr
        psot = 12 + len(hdr) + 2 + len(data)
        body += struct.pack(">HHHIBB", 0xFF90, 10, t, psot, 0, 1) + hdr + b"\xff\x93" + data
        lens.append((t, psot))
    head = b"\xff\x4f" + b"".join(s for m, s in a_segs if m != 0xFF55)
    if tlm:
        head += _seg(0xFF55, bytes([0, 0x60]) + b"".join(struct.pack(">HI", t, n) for t, n in lens))
    return head + body + b"\xff\xd9"


# name -> (H, W, base keywords A, tile keywords B, B tiles, form); every case 3 components of 8 bits
TILES = (48, 40)
CASES = {
    "levels_cblk": (80, 96, dict(numres=3), dict(numres=5, cblk=(32, 32)), {1, 2}, "cod"),
    "rev_to_irrev": (80, 96, dict(numres=4), dict(numres=4, irreversible=True), {0, 3}, "cod"),
    "coc_form": (80, 96, dict(numres=4), dict(numres=3, cblk=(16, 16), precincts=[(16, 16)]), {1, 3}, "coc"),
    "prog_layers_sop": (80, 96, dict(numres=3), dict(numres=4, nlayers=3, prog_order="RPCL", sop=True, eph=True),
                        {2}, "cod"),
    "ht_tile": (80, 96, dict(numres=4), dict(numres=4, cblk_sty=0x40), {0, 1}, "cod"),
    "modes_tile": (80, 96, dict(numres=3, cblk=(32, 32)), dict(numres=3, cblk_sty=0x05), {3}, "cod"),
    "scope_irrev": (80, 96, dict(numres=3), dict(numres=3, irreversible=True), {1, 2}, "scope"),
    "ragged_tiles": (70, 101, dict(numres=3), dict(numres=2, cblk=(16, 16)), {2, 5}, "cod"),
    "roi_tile": (80, 96, dict(numres=3), dict(numres=3, roi=(1, 9)), {0, 3}, "rgn"),
}
# an image area off the canvas origin, tile grid at (0, 0): the first tiles are clipped
CASES["origin_tiles"] = (75, 90, dict(numres=3, origin=(13, 7), tile_origin=(0, 0)),
                         dict(numres=4, cblk=(16, 16), origin=(13, 7), tile_origin=(0, 0)), {0, 4}, "cod")


def image(name):
    import numpy as np
    H, W = CASES[name][:2]
    rng = np.random.default_rng(sum(map(ord, name)))
    yy, xx = np.mgrid[0:H, 0:W]
    return np.stack([((xx * (c + 2) + yy * 3 + rng.integers(0, 24, size=(H, W))) % 256) for c in range(3)]).astype(np.int32)


def encodes(name):
    H, W, ka, kb, tiles, form = CASES[name]
    img = image(name)
    return O.encode(img, 8, tiles=TILES, **ka), O.encode(img, 8, tiles=TILES, **kb)


def stream(name, tlm=False):
    H, W, ka, kb, tiles, form = CASES[name]
    a, b = encodes(name)
    return splice(a, b, tiles, form, tlm=tlm)


def tile_rects(name):
    """{tile: (x0, y0, x1, y1)} of the case's tile grid in image coordinates (B.3: the tiles of the
    grid at the canvas origin, clipped to the image area)."""
    H, W, ka = CASES[name][:3]
    ox, oy = ka.get("origin") or (0, 0)
    tw, th = TILES
    nx, ny = -(-(ox + W) // tw), -(-(oy + H) // th)
    out = {}
    for t in range(nx * ny):
        i, j = t % nx, t // nx
        out[t] = (max(i * tw, ox) - ox, max(j * th, oy) - oy, min(ox + W, (i + 1) * tw) - ox, min(oy + H, (j + 1) * th) - oy)
    return out


def expected(name, partial=False, reduce=0):
    """A's decode with B's on the B tiles (each tile decodes on its own)."""
    a, b = encodes(name)
    O.set_decode_reduce(reduce)
    try:
        da, _ = O.decode(a, partial=partial)
        db, _ = O.decode(b, partial=partial)
    finally:
        O.set_decode_reduce(0)
    out = da.copy()
    r = 1 << reduce
    ox, oy = CASES[name][2].get("origin") or (0, 0)
    cx = lambda v: -(-(v + ox) // r) - -(-ox // r)   # (reduced canvas edges, less the image origin's)
    cy = lambda v: -(-(v + oy) // r) - -(-oy // r)
    for t, (x0, y0, x1, y1) in tile_rects(name).items():
        if t in CASES[name][4]:
            out[:, cy(y0):cy(y1), cx(x0):cx(x1)] = db[:, cy(y0):cy(y1), cx(x0):cx(x1)]
    return out
