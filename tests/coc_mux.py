"""Codestreams whose components are coded with different parameters (COC / QCC markers), made by
multiplexing single-component oracle streams.

Neither Grok's encoder nor the oracle's writes a COC (grk_cparameters has one coding style for
every component), and Pillow exposes no such option, so test streams are assembled: each component
is encoded alone by the oracle (LRCP, one tile, PLT giving every packet's length), and the packets
are interleaved in the multi-component LRCP order (layer, resolution, component, precinct;
A.6.1 / B.12.1.1), a component without resolution r contributing none there.  The main header
takes component 0's COD (MCT off) and QCD, and a COC / QCC for every other component whose coding /
quantisation differs (A.6.2, A.6.5).  Each component's packets are unchanged, so a decoder must
reproduce each single-component decode; OpenJPEG 2.5.4 does (tests/test_coc.py)."""
import os
import struct
import sys

from conftest import ROOT

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402


def _markers(cs):
    """Main-header markers {code: body} (first of each) and the tile part's (PLT lengths, data)."""
    i, main = 2, {}
    while True:
        m, L = struct.unpack(">HH", cs[i:i + 4])
        if m == 0xFF90:
            break
        main.setdefault(m, cs[i + 4:i + 2 + L])
        i += 2 + L
    sot = i
    psot = struct.unpack(">I", cs[sot + 6:sot + 10])[0]
    j, plt = sot + 12, []
    while struct.unpack(">H", cs[j:j + 2])[0] != 0xFF93:
        m, L = struct.unpack(">HH", cs[j:j + 4])
        if m == 0xFF58:
            v = 0
            for b in cs[j + 5:j + 2 + L]:
                v = (v << 7) | (b & 0x7F)
                if not b & 0x80:
                    plt.append(v)
                    v = 0
        j += 2 + L
    data = cs[j + 2:sot + psot]
    assert sum(plt) == len(data)
    return main, plt, data


def _nprc(w, h, numres, prc):
    """Packets per resolution of a one-tile image at the origin (precinct exponents per resolution)."""
    out = []
    for r in range(numres):
        lv = numres - 1 - r
        rx1, ry1 = -(-w >> lv), -(-h >> lv)
        pw, ph = prc[r]
        out.append(((-(-rx1 >> pw)) * (-(-ry1 >> ph))) if rx1 and ry1 else 0)
    return out


def _prc_exps(cod):
    numres = cod[5] + 1
    if cod[0] & 1:
        return [(cod[10 + r] & 15, cod[10 + r] >> 4) for r in range(numres)]
    return [(15, 15)] * numres


def mux(planes, prec, comp_kw, nlayers=1):
    """planes: list of (H, W) int32 arrays (one size); prec: the precision, or one per component
    (SIZ Ssiz; the QCD / QCC follow it); comp_kw: per component oracle.encode keyword arguments
    (numres, cblk, irreversible, cblk_sty, precincts, layer_rate ...).
    Returns the multi-component codestream."""
    h, w = planes[0].shape
    precs = list(prec) if isinstance(prec, (list, tuple)) else [prec] * len(planes)
    parts = []
    for p, kw, pr in zip(planes, comp_kw, precs):
        kw = dict(kw, plt=True, mct=False, write_com=False)
        if "layer_rate" not in kw:
            kw["nlayers"] = nlayers
        cs = O.encode(p[None], pr, **kw)
        main, plt, data = _markers(cs)
        cod = main[0xFF52]
        assert cod[1] == 0 and struct.unpack(">H", cod[2:4])[0] == nlayers   # LRCP, the same layers
        npr = _nprc(w, h, cod[5] + 1, _prc_exps(cod))
        # packets in (layer, resolution, precinct) order -> {(l, r): bytes}
        pk, k, off = {}, 0, 0
        for l in range(nlayers):
            for r, n in enumerate(npr):
                b = b""
                for _ in range(n):
                    b += data[off:off + plt[k]]
                    off += plt[k]
                    k += 1
                pk[(l, r)] = b
        assert k == len(plt)
        parts.append((main, cod, npr, pk))
    nc = len(planes)
    siz0 = parts[0][0][0xFF51]
    siz = bytearray(siz0[:34]) + struct.pack(">H", nc) + b"".join(bytes([pr - 1, 1, 1]) for pr in precs)
    cod0 = bytearray(parts[0][1])
    cod0[4] = 0   # no MCT
    o = bytearray(b"\xff\x4f")
    o += struct.pack(">HH", 0xFF51, 2 + len(siz)) + siz
    o += struct.pack(">HH", 0xFF52, 2 + len(cod0)) + cod0
    qcd0 = parts[0][0][0xFF5C]
    o += struct.pack(">HH", 0xFF5C, 2 + len(qcd0)) + qcd0
    for c in range(1, nc):
        cod = parts[c][1]
        coc = bytes([c, cod[0] & 1]) + cod[5:]
        if coc[1:] != bytes([cod0[0] & 1]) + bytes(cod0[5:]):
            o += struct.pack(">HH", 0xFF53, 2 + len(coc)) + coc
        qcd = parts[c][0][0xFF5C]
        if qcd != qcd0:
            o += struct.pack(">HH", 0xFF5D, 3 + len(qcd)) + bytes([c]) + qcd
    body = b""
    nres = max(len(p[2]) for p in parts)
    for l in range(nlayers):
        for r in range(nres):
            for c in range(nc):
                if r < len(parts[c][2]):
                    body += parts[c][3][(l, r)]
    sot = struct.pack(">HHHIBB", 0xFF90, 10, 0, 12 + 2 + len(body), 0, 1)
    o += sot + b"\xff\x93" + body + b"\xff\xd9"
    return bytes(o)
