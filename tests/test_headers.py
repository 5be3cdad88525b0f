"""Host-side codestream logic without a GPU: header validation of untrusted streams
(gk_probe_header, the parse behind grk_decompress_read_header), the JP2 file-format
boxes, and the oracle's threaded / tile-part paths used by the full-size fixtures."""
import hashlib
import struct

import numpy as np
import pytest

import grok_amd as G
import oracle as O
from conftest import FIXTURES
from grok_amd.synth import synth_image


def _stream():
    return next(f for f in FIXTURES if f.name == "rgb8_64").cs


def _patch(cs, marker, off, val, fmt=">B"):
    """Overwrite a field `off` bytes into the segment of the first `marker` of the main header."""
    b = bytearray(cs)
    i = 2
    while i + 4 <= len(b):
        m, L = struct.unpack(">HH", b[i:i + 4])
        if m == marker:
            struct.pack_into(fmt, b, i + 4 + off, val)
            return bytes(b)
        i += 2 + L
    raise AssertionError("marker not found")


def test_probe_reads_fixture_header():
    for f in FIXTURES:
        info = G.probe_header(f.cs)
        c, h, w = f.img.shape
        assert (info.w, info.h, info.numcomps, info.prec) == (w, h, c, f.bits)


@pytest.mark.parametrize("mutate,msg", [
    (lambda cs: cs[:30], "incomplete|corrupt"),                                  # truncated main header
    (lambda cs: b"\x00\x01" + cs[2:], "SOC"),                                    # not a codestream
    (lambda cs: _patch(cs, 0xFF52, 5, 40), "decomposition"),                     # COD: 41 resolutions
    (lambda cs: _patch(cs, 0xFF51, 36, 0x7F), "precision"),                      # SIZ: 128-bit samples
    (lambda cs: _patch(cs, 0xFF51, 34, 0, ">H"), "component count"),             # SIZ: no components
    (lambda cs: _patch(cs, 0xFF5C, -2, 2, ">H"), "QCD|marker length|corrupt"),   # QCD: Lqcd = 2
    (lambda cs: _patch(cs, 0xFF52, 6, 9), "code-block"),                         # COD: 2^11 wide blocks
    (lambda cs: _patch(cs, 0xFF51, -2, 0xFFF0, ">H"), "marker length|corrupt"),  # SIZ length past the end
])
def test_probe_rejects_malformed_headers(mutate, msg):
    with pytest.raises(ValueError, match=msg):
        G.probe_header(mutate(_stream()))


def _boxes(b):
    out, pos = [], 0
    while pos + 8 <= len(b):
        L, T = struct.unpack(">I4s", b[pos:pos + 8])
        hdr = 8
        if L == 1:
            L = struct.unpack(">Q", b[pos + 8:pos + 16])[0]
            hdr = 16
        elif L == 0:
            L = len(b) - pos
        out.append((T.decode(), pos, hdr, L))
        pos += L
    return out


def test_jp2_layout_oracle():
    # FileFormatCompress: jP, ftyp, jp2h{ihdr, colr}, jp2c (8-byte header below 2^30 raw bytes)
    img = synth_image(48, 80, 3, 8, 3).astype(np.int32)
    raw = O.encode(img, 8)
    jp2 = O.encode(img, 8, jp2=True)
    assert jp2.endswith(raw)
    bx = _boxes(jp2)
    assert [t for t, *_ in bx] == ["jP  ", "ftyp", "jp2h", "jp2c"]
    assert jp2[8:12] == b"\x0d\x0a\x87\x0a" and jp2[16:20] == b"ftyp" and jp2[20:24] == b"jp2 "
    ihdr = jp2[bx[2][1] + 8:]
    assert ihdr[4:8] == b"ihdr" and struct.unpack(">IIHBBBB", ihdr[8:22]) == (48, 80, 3, 7, 7, 0, 0)
    colr = ihdr[22:37]
    assert colr[4:8] == b"colr" and colr[8] == 1 and struct.unpack(">I", colr[11:15])[0] == 16   # sRGB
    t, pos, hdr, L = bx[3]
    assert hdr == 8 and L == 8 + len(raw)
    # greyscale enumeration for one component; XL box once the raw image passes 2^30 bytes
    g = O.jp2_header(100, 100, 1, 8, 1234)
    assert struct.unpack(">I", g[-12:-8])[0] == 17 and struct.unpack(">I", g[-8:-4])[0] == 1234 + 8
    big = O.jp2_header(32768, 32768, 3, 8, 10)
    assert len(big) == len(g) + 8 and struct.unpack(">I4sQ", big[-16:]) == (1, b"jp2c", 10 + 16)
    # the decoders find the codestream inside the file
    d, _ = O.decode(jp2)
    np.testing.assert_array_equal(d, img)
    info = G.probe_header(jp2)
    assert (info.w, info.h, info.numcomps, info.prec) == (80, 48, 3, 8)


def test_probe_rejects_bad_jp2():
    img = synth_image(16, 16, 1, 8, 3).astype(np.int32)
    jp2 = bytearray(O.encode(img, 8, jp2=True))
    bad = bytes(jp2[:12]) + bytes(jp2[32:])            # no ftyp box
    with pytest.raises(ValueError, match="file type"):
        G.probe_header(bad)
    with pytest.raises(ValueError, match="codestream box|length"):
        G.probe_header(bytes(jp2[:77]))                  # cut before the jp2c box


def test_oracle_threads_do_not_change_output():
    img = synth_image(200, 264, 3, 8, 9).astype(np.int32)
    outs = []
    for th in (1, 3, 8):
        O.set_threads(th)
        outs.append(O.encode(img, 8, tiles=(64, 64), tlm=True, plt=True))
        outs.append(O.encode(img, 8))
    O.set_threads(1)
    assert outs[0] == outs[2] == outs[4] and outs[1] == outs[3] == outs[5]


def test_oracle_tile_parts_assemble_to_full_encode():
    # the C5 fixture path: tile rows coded from slabs, assembled under the main header + TLM
    H, W, th = 200, 264, 64
    img = synth_image(H, W, 3, 8, 9).astype(np.int32)
    kw = dict(tiles=(64, th), tlm=True, plt=True)
    full = O.encode(img, 8, jp2=True, **kw)
    hdr, tlm = O.main_header(W, H, 3, 8, **kw)
    ntx = (W + 63) // 64
    body, lens = b"", []
    for j in range(0, (H + th - 1) // th):
        y0, y1 = j * th, min(H, (j + 1) * th)
        b, ln = O.encode_tile_parts(img[:, y0:y1], y0, (H, W), 8, j * ntx, (j + 1) * ntx, **kw)
        body += b
        lens += ln
    h = bytearray(hdr)
    for t, n in enumerate(lens):
        h[tlm + 6 * t:tlm + 6 * t + 6] = struct.pack(">HI", t, n)
    cs = bytes(h) + body + b"\xff\xd9"
    assert O.jp2_header(W, H, 3, 8, len(cs)) + cs == full
    assert hashlib.sha256(cs).digest() == hashlib.sha256(O.encode(img, 8, **kw)).digest()
