"""Codestream edits for the COC / QCC / tile-part COD / QCD tests (ISO 15444-1 A.6.2, A.6.5).

Builds marker segments that restate (or change) the main header's COD / QCD for one component
or one tile and splices them into a codestream: main-header markers go in front of the first
SOT; tile-part markers go after the first SOT (Psot, and the first TLM entry when present,
grow by the inserted length).
"""


def main_markers(cs):
    """[(offset, code, Lmarker)] of the main header, SOC excluded, up to the first SOT."""
    out, i = [], 2
    while True:
        m = int.from_bytes(cs[i:i + 2], "big")
        if m == 0xff90:
            return out, i
        L = int.from_bytes(cs[i + 2:i + 4], "big")
        out.append((i, m, L))
        i += 2 + L


def body(cs, code):
    ms, _ = main_markers(cs)
    o, _, L = next(x for x in ms if x[1] == code)
    return bytes(cs[o + 4:o + 2 + L])


def ncomp(cs):
    return int.from_bytes(body(cs, 0xff51)[34:36], "big")


def segment(code, payload):
    return code.to_bytes(2, "big") + (len(payload) + 2).to_bytes(2, "big") + payload


def coc(cs, comp, sty_xor=0):
    """COC for `comp` restating COD's Scod precinct flag and SPcod (code-block style ^ sty_xor)."""
    cod = bytearray(body(cs, 0xff52))
    cod[8] ^= sty_xor
    cw = 1 if ncomp(cs) <= 256 else 2
    return segment(0xff53, comp.to_bytes(cw, "big") + bytes([cod[0] & 1]) + bytes(cod[5:]))


def qcc(cs, comp, guard_add=0):
    """QCC for `comp` restating QCD (guard-bit count + guard_add)."""
    q = bytearray(body(cs, 0xff5c))
    q[0] = (q[0] + (guard_add << 5)) & 0xff
    cw = 1 if ncomp(cs) <= 256 else 2
    return segment(0xff5d, comp.to_bytes(cw, "big") + bytes(q))


def rgn(cs, comp, shift):
    """RGN for `comp`: implicit (maxshift) style, ROI shift `shift` (A.6.3)."""
    cw = 1 if ncomp(cs) <= 256 else 2
    return segment(0xff5e, comp.to_bytes(cw, "big") + bytes([0, shift]))


def cod(cs, layers_add=0):
    b = bytearray(body(cs, 0xff52))
    n = int.from_bytes(b[2:4], "big") + layers_add
    b[2:4] = n.to_bytes(2, "big")
    return segment(0xff52, bytes(b))


def qcd(cs):
    return segment(0xff5c, body(cs, 0xff5c))


def insert_main(cs, segs):
    _, sot = main_markers(cs)
    return cs[:sot] + segs + cs[sot:]


def insert_tile_part(cs, segs):
    """Put `segs` into the first tile-part header; fix its Psot and its TLM entry."""
    ms, sot = main_markers(cs)
    n = len(segs)
    out = bytearray(cs)
    psot = int.from_bytes(cs[sot + 6:sot + 10], "big")
    if psot:
        out[sot + 6:sot + 10] = (psot + n).to_bytes(4, "big")
    for o, m, L in ms:
        if m == 0xff55:   # TLM: Ztlm, Stlm, then (Ttlm, Ptlm) entries; the first is this tile part
            stlm = cs[o + 5]
            st, sp = (stlm >> 4) & 3, (stlm >> 6) & 1
            e, w = o + 6 + st, 4 if sp else 2
            out[e:e + w] = (int.from_bytes(cs[e:e + w], "big") + n).to_bytes(w, "big")
            break
    return bytes(out[:sot + 12]) + segs + bytes(out[sot + 12:])
