"""ctypes wrapper for the CPU oracle (oracle/j2k_oracle.cpp).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and the
cpu_baseline leg of bench.py, as the checker.  The product (grok_amd) never
imports this module.
"""
import ctypes
import os

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "libj2k_oracle.so")
_lib = None


class CParams(ctypes.Structure):
    _fields_ = [
        ("numres", ctypes.c_uint32), ("cbw_exp", ctypes.c_uint32), ("cbh_exp", ctypes.c_uint32),
        ("irreversible", ctypes.c_uint32), ("mct", ctypes.c_uint32), ("nlayers", ctypes.c_uint32),
        ("write_com", ctypes.c_uint32),
        ("prcw_exp", ctypes.c_uint32 * 33), ("prch_exp", ctypes.c_uint32 * 33),
        ("layer_rate", ctypes.c_double * 100),
        ("cblk_sty", ctypes.c_uint32),
        ("tile_w", ctypes.c_uint32), ("tile_h", ctypes.c_uint32), ("tlm", ctypes.c_uint32), ("plt", ctypes.c_uint32),
        ("cod_format", ctypes.c_uint32), ("prog_order", ctypes.c_uint32), ("tp_div", ctypes.c_uint32),
        ("numpocs", ctypes.c_uint32), ("pocs", (ctypes.c_uint32 * 6) * 32),
        ("roi_compno", ctypes.c_int32), ("roi_shift", ctypes.c_uint32),
        ("csty", ctypes.c_uint32), ("by_quality", ctypes.c_uint32), ("layer_distortion", ctypes.c_double * 100),
        ("image_x0", ctypes.c_uint32), ("image_y0", ctypes.c_uint32), ("tile_x0", ctypes.c_uint32),
        ("tile_y0", ctypes.c_uint32),
        ("nq", ctypes.c_uint32), ("comp_gb", ctypes.c_uint32 * 16), ("comp_qshift", ctypes.c_int32 * 16),
        ("qderived", ctypes.c_uint32),
        ("nsub", ctypes.c_uint32), ("sub_dx", ctypes.c_uint32 * 16), ("sub_dy", ctypes.c_uint32 * 16),
        ("ppx", ctypes.c_uint32),
        ("ncom", ctypes.c_uint32), ("com_data", ctypes.c_char_p), ("com_len", ctypes.c_uint32 * 16),
        ("com_binary", ctypes.c_uint32 * 16),
    ]


class Block(ctypes.Structure):
    _fields_ = [(n, ctypes.c_uint32) for n in
                ("comp", "res", "band", "prc", "cblk", "x0", "y0", "x1", "y1", "numbps", "npasses", "len")] + \
               [("data_off", ctypes.c_uint64)]


def build():
    """Compile the oracle with its Makefile (gcc only)."""
    import subprocess
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_LIB_PATH):
            build()
        _lib = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER
        _lib.orc_encode.restype = ctypes.c_size_t
        _lib.orc_encode.argtypes = [P(ctypes.c_int32), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                    ctypes.c_uint32, ctypes.c_int, P(CParams), ctypes.c_void_p, ctypes.c_size_t]
        _lib.orc_decode.restype = ctypes.c_int
        _lib.orc_decode.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p] + [P(ctypes.c_uint32)] * 4
        _lib.orc_set_partial.argtypes = [ctypes.c_int]
        _lib.orc_last_comp_dims.restype = ctypes.c_uint32
        _lib.orc_last_comp_dims.argtypes = [ctypes.c_void_p]
        _lib.orc_last_comp_prec.restype = ctypes.c_uint32
        _lib.orc_last_comp_prec.argtypes = [ctypes.c_void_p]
        _lib.orc_inv53_single.argtypes = [ctypes.c_int32, ctypes.c_uint32, ctypes.c_int, ctypes.c_int]
        _lib.orc_inv53_single.restype = ctypes.c_int32
        _lib.orc_forward_coefs.argtypes = [P(ctypes.c_int32), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_int, P(CParams), P(ctypes.c_int32)]
        _lib.orc_encode_blocks.argtypes = [P(ctypes.c_int32), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                           ctypes.c_uint32, ctypes.c_int, P(CParams), ctypes.c_void_p,
                                           P(ctypes.c_uint32), ctypes.c_void_p, P(ctypes.c_uint64)]
        _lib.orc_encode_block_passes.argtypes = [P(ctypes.c_int32), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                                 ctypes.c_uint32, ctypes.c_int, P(CParams), ctypes.c_void_p,
                                                 ctypes.c_void_p, P(ctypes.c_uint64)]
        _lib.orc_t1_encode_cblk.restype = ctypes.c_int
        _lib.orc_t1_encode_cblk.argtypes = [P(ctypes.c_int32)] + [ctypes.c_uint32] * 4 + [
            ctypes.c_void_p, ctypes.c_uint32, P(ctypes.c_uint32), P(ctypes.c_uint32), ctypes.c_void_p, ctypes.c_void_p]
        _lib.orc_t1_decode_cblk.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 6 + [P(ctypes.c_int32)]
        _lib.orc_default_params.argtypes = [P(CParams)]
        _lib.orc_set_threads.argtypes = [ctypes.c_uint]
        _lib.orc_get_threads.restype = ctypes.c_uint
        _lib.orc_jp2_header.restype = ctypes.c_size_t
        _lib.orc_jp2_header.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p]
        _lib.orc_main_header.restype = ctypes.c_size_t
        _lib.orc_main_header.argtypes = [ctypes.c_uint32] * 4 + [ctypes.c_int, P(CParams), ctypes.c_void_p,
                                                                ctypes.c_size_t, P(ctypes.c_size_t)]
        _lib.orc_encode_tile_parts.restype = ctypes.c_size_t
        _lib.orc_encode_tile_parts.argtypes = [ctypes.c_void_p] + [ctypes.c_uint32] * 4 + [ctypes.c_int, P(CParams)] + \
            [ctypes.c_uint32] * 4 + [ctypes.c_void_p, ctypes.c_size_t, P(ctypes.c_uint32)]
        _lib.orc_ht_encode_cblk.restype = ctypes.c_int
        _lib.orc_ht_encode_cblk.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_void_p, ctypes.c_uint32]
        _lib.orc_ht_decode_cblk.restype = ctypes.c_int
        _lib.orc_ht_decode_cblk.argtypes = [ctypes.c_void_p, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint32,
                                            ctypes.c_uint32, ctypes.c_void_p]
    return _lib


def set_threads(n):
    """Worker threads for code-blocks / tiles (results do not depend on the count)."""
    lib().orc_set_threads(int(n))


def get_threads():
    return int(lib().orc_get_threads())


def params(numres=6, cblk=(64, 64), irreversible=False, mct=True, nlayers=1, write_com=True, precincts=None,
           layer_rate=None, cblk_sty=0, tiles=None, tlm=False, plt=False, jp2=False, prog_order=0, tile_parts=None, pocs=None, roi=None,
           sop=False, eph=False, quality=None, origin=None, tile_origin=None, comp_guard_bits=None, comp_qshift=None,
           qderived=False, subsampling=None, packed_headers=None, comments=None):
    p = CParams()
    lib().orc_default_params(ctypes.byref(p))
    p.numres = numres
    p.cbw_exp = int(cblk[0]).bit_length() - 1
    p.cbh_exp = int(cblk[1]).bit_length() - 1
    p.irreversible = int(irreversible)
    p.mct = int(mct)
    p.nlayers = nlayers
    p.write_com = int(write_com)
    p.cblk_sty = int(cblk_sty)
    p.prog_order = ["LRCP", "RLCP", "RPCL", "PCRL", "CPRL"].index(prog_order) if isinstance(prog_order, str) \
        else int(prog_order)
    p.tp_div = ord(tile_parts) if tile_parts else 0
    progs = ["LRCP", "RLCP", "RPCL", "PCRL", "CPRL"]
    for i, e in enumerate(pocs or []):
        p.pocs[i][:] = list(e[:5]) + [progs.index(e[5]) if isinstance(e[5], str) else int(e[5])]
    p.numpocs = len(pocs or [])
    p.roi_compno, p.roi_shift = (int(roi[0]), int(roi[1])) if roi else (-1, 0)
    if tiles:
        p.tile_w, p.tile_h = int(tiles[0]), int(tiles[1])
    # canvas offsets: image area at origin (grk_compress -d), tile grid at tile_origin (-T; -T alone
    # also moves the image origin there, grk_compress.cpp:1547-1551)
    if tile_origin:
        p.tile_x0, p.tile_y0 = int(tile_origin[0]), int(tile_origin[1])
    if origin:
        p.image_x0, p.image_y0 = int(origin[0]), int(origin[1])
    elif tile_origin:
        p.image_x0, p.image_y0 = p.tile_x0, p.tile_y0
    p.tlm, p.plt = int(tlm), int(plt)
    # per-component quantisation, written as QCC markers (third-party encoders; Grok writes none)
    if comp_guard_bits or comp_qshift:
        n = max(len(comp_guard_bits or []), len(comp_qshift or []))
        p.nq = n
        for c in range(n):
            p.comp_gb[c] = int((comp_guard_bits or [])[c]) if c < len(comp_guard_bits or []) else 2
            p.comp_qshift[c] = int((comp_qshift or [])[c]) if c < len(comp_qshift or []) else 0
    p.qderived = int(bool(qderived))
    # component subsampling [(dx, dy), ...] (grk_image_comp::dx / dy; SIZ XRsiz / YRsiz)
    if subsampling:
        p.nsub = len(subsampling)
        for c, (dx, dy) in enumerate(subsampling):
            p.sub_dx[c], p.sub_dy[c] = int(dx), int(dy)
    # caller comments (grk_compress -C): [str (text) or bytes (binary)], written instead of the default
    if comments:
        bufs = [c if isinstance(c, bytes) else c.encode() for c in comments]
        p._com = b"".join(bufs)
        p.ncom = len(bufs)
        p.com_data = p._com
        for i, (b, c) in enumerate(zip(bufs, comments)):
            p.com_len[i], p.com_binary[i] = len(b), int(isinstance(c, bytes))
    # packed packet headers: "ppt" (tile-part headers) or "ppm" (main header); test streams only
    p.ppx = {None: 0, "ppt": 1, "ppm": 2}[packed_headers]
    p.cod_format = 2 if jp2 else 0
    if layer_rate:
        p.nlayers = len(layer_rate)
        for i, r in enumerate(layer_rate):
            p.layer_rate[i] = r
    # grk_compress -S / -E (csty SOP / EPH bits) and -q PSNR layers (allocationByQuality)
    p.csty = (2 if sop else 0) | (4 if eph else 0)
    if quality:
        p.by_quality = 1
        p.nlayers = len(quality)
        for i, q in enumerate(quality):
            p.layer_distortion[i] = q
    if precincts:
        # Grok CLI semantics (CodeStreamCompress.cpp:542-590): sizes from the highest resolution
        # down; past the list, the last size shifted right once per resolution; a size below 1
        # takes exponent 1, any other floorlog2(size) -- so a shift that reaches exactly 1 gives
        # exponent 0 (1 x 1 code-blocks at resolution 0)
        def _exp(s):
            return 1 if s < 1 else int(s).bit_length() - 1
        ns = len(precincts)
        for k in range(numres):
            r = numres - 1 - k
            if k < ns:
                w, h = precincts[k]
            else:
                w, h = precincts[-1][0] >> (k - (ns - 1)), precincts[-1][1] >> (k - (ns - 1))
            p.prcw_exp[r], p.prch_exp[r] = _exp(int(w)), _exp(int(h))
    return p


def _planes(img):
    """img: (C, H, W) int32 array -> contiguous int32 planes."""
    a = np.ascontiguousarray(img, dtype=np.int32)
    assert a.ndim == 3
    return a


def comp_shape(w, h, dx, dy, origin=(0, 0)):
    """(rows, cols) of a component sampled every (dx, dy) on the canvas (grk_image_comp h / w)."""
    x0, y0 = origin
    return -(-(y0 + h) // dy) - -(-y0 // dy), -(-(x0 + w) // dx) - -(-x0 // dx)


def encode(img, prec, signed=False, size=None, **kw):
    """img: (C, H, W) int32 array; with subsampling=[(dx, dy), ...], a list of per-component 2-D
    planes of comp_shape(W, H, dx, dy, origin) and size=(W, H), the image area."""
    if kw.get("subsampling"):
        planes = [np.ascontiguousarray(x, dtype=np.int32) for x in img]
        w, h = size
        c = len(planes)
        for k, (dx, dy) in enumerate(kw["subsampling"]):
            assert planes[k].shape == comp_shape(w, h, dx, dy, kw.get("origin") or (0, 0)), (k, planes[k].shape)
        a = np.concatenate([x.ravel() for x in planes])
    else:
        a = _planes(img)
        c, h, w = a.shape
    p = params(**kw)
    cap = a.nbytes * 2 + (1 << 16)
    out = np.empty(cap, dtype=np.uint8)
    n = lib().orc_encode(a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), w, h, c, prec, int(signed),
                         ctypes.byref(p), out.ctypes.data, cap)
    if n == 0:
        raise RuntimeError("oracle encode failed")
    return out[:n].tobytes()


def jp2_header(w, h, nc, prec, cs_len, signed=False):
    """JP2 boxes in front of a codestream of cs_len bytes (file = header + codestream)."""
    buf = np.empty(128, np.uint8)
    n = lib().orc_jp2_header(w, h, nc, prec, int(signed), cs_len, buf.ctypes.data)
    return buf[:n].tobytes()


def main_header(w, h, nc, prec, signed=False, **kw):
    """(main header bytes, TLM entry offset or 0) for assembling separately coded tile parts."""
    p = params(**kw)
    buf = np.empty(1 << 20, np.uint8)
    tlm = ctypes.c_size_t()
    n = lib().orc_main_header(w, h, nc, prec, int(signed), ctypes.byref(p), buf.ctypes.data, buf.size,
                              ctypes.byref(tlm))
    if n == 0:
        raise RuntimeError("oracle main header failed")
    return buf[:n].tobytes(), tlm.value


def encode_tile_parts(slab, row0, image_hw, prec, tile_begin, tile_end, signed=False, **kw):
    """Tile parts of tiles [tile_begin, tile_end) from a (C, rows, W) slab holding image rows
    [row0, row0 + rows).  Returns (bytes, [Psot per tile])."""
    a = _planes(slab)
    c, rows, w = a.shape
    H, W = image_hw
    assert W == w
    p = params(**kw)
    cap = a.nbytes * 2 + (1 << 20)
    out = np.empty(cap, np.uint8)
    lens = (ctypes.c_uint32 * (tile_end - tile_begin))()
    n = lib().orc_encode_tile_parts(a.ctypes.data, W, H, c, prec, int(signed), ctypes.byref(p), row0, rows,
                                    tile_begin, tile_end, out.ctypes.data, cap, lens)
    if n == 0:
        raise RuntimeError("oracle tile-part encode failed")
    return out[:n].tobytes(), list(lens)


def set_decode_layers(n):
    """Decode only the first n quality layers from now on (0 = all; grk_decompress -l)."""
    lib().orc_set_decode_layers(ctypes.c_uint32(int(n)))


def set_decode_reduce(n):
    """Discard the n highest resolutions from now on (grk_decompress -r / cp_reduce)."""
    lib().orc_set_decode_reduce(ctypes.c_uint32(int(n)))


def decode(cs, partial=False):
    """Decode the whole image.  partial: as Grok decodes once a window is set (its partial-tile
    inverse for every tile, which shifts a single odd 5/3 sample across instead of halving it);
    crop the result to the window."""
    buf = np.frombuffer(cs, dtype=np.uint8).copy()
    buf = np.concatenate([buf, np.zeros(8, np.uint8)])
    W, H, NC, PREC = (ctypes.c_uint32() for _ in range(4))
    rc = lib().orc_decode(buf.ctypes.data, len(cs), None, ctypes.byref(W), ctypes.byref(H), ctypes.byref(NC),
                          ctypes.byref(PREC))
    if rc != 0:
        raise RuntimeError("oracle decode header failed: %d" % rc)
    dims = (ctypes.c_uint32 * (2 * NC.value))()
    lib().orc_last_comp_dims(dims)
    shapes = [(dims[2 * c + 1], dims[2 * c]) for c in range(NC.value)]
    flat = np.empty(sum(a * b for a, b in shapes), dtype=np.int32)
    lib().orc_set_partial(int(bool(partial)))
    try:
        rc = lib().orc_decode(buf.ctypes.data, len(cs), flat.ctypes.data, ctypes.byref(W), ctypes.byref(H),
                              ctypes.byref(NC), ctypes.byref(PREC))
    finally:
        lib().orc_set_partial(0)
    if rc != 0:
        raise RuntimeError("oracle decode failed: %d" % rc)
    if all(sh == (H.value, W.value) for sh in shapes):
        return flat.reshape(NC.value, H.value, W.value), PREC.value
    # subsampled components: one plane each, at its own size
    out, o = [], 0
    for sh in shapes:
        out.append(flat[o:o + sh[0] * sh[1]].reshape(sh))
        o += sh[0] * sh[1]
    return out, PREC.value


def last_comp_prec():
    """[(precision, signed)] per component of the last decode (SIZ Ssiz)."""
    n = lib().orc_last_comp_prec(None)
    v = (ctypes.c_uint32 * max(n, 1))()
    lib().orc_last_comp_prec(v)
    return [(v[c] & 0xff, bool(v[c] >> 8)) for c in range(n)]


def forward_coefs(img, prec, signed=False, **kw):
    a = _planes(img)
    c, h, w = a.shape
    p = params(**kw)
    out = np.empty_like(a)
    lib().orc_forward_coefs(a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), w, h, c, prec, int(signed),
                            ctypes.byref(p), out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


def encode_blocks(img, prec, signed=False, **kw):
    """Per-block T1 results in canonical (comp, res, band, precinct, cblk) order."""
    a = _planes(img)
    c, h, w = a.shape
    p = params(**kw)
    nb = ctypes.c_uint32()
    nbytes = ctypes.c_uint64()
    ip = a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    lib().orc_encode_blocks(ip, w, h, c, prec, int(signed), ctypes.byref(p), None, ctypes.byref(nb), None,
                            ctypes.byref(nbytes))
    blocks = (Block * nb.value)()
    data = np.empty(max(1, nbytes.value), dtype=np.uint8)
    lib().orc_encode_blocks(ip, w, h, c, prec, int(signed), ctypes.byref(p), blocks, ctypes.byref(nb),
                            data.ctypes.data, ctypes.byref(nbytes))
    return blocks, data[:nbytes.value]


def encode_block_passes(img, prec, signed=False, **kw):
    """Pass rates (uint32) and cumulative distortion decreases (float64) of every code-block,
    concatenated in encode_blocks order (each block contributes its npasses entries)."""
    a = _planes(img)
    c, h, w = a.shape
    p = params(**kw)
    n = ctypes.c_uint64()
    ip = a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))
    lib().orc_encode_block_passes(ip, w, h, c, prec, int(signed), ctypes.byref(p), None, None, ctypes.byref(n))
    rates = np.zeros(max(1, n.value), np.uint32)
    dists = np.zeros(max(1, n.value), np.float64)
    lib().orc_encode_block_passes(ip, w, h, c, prec, int(signed), ctypes.byref(p), rates.ctypes.data,
                                  dists.ctypes.data, ctypes.byref(n))
    return rates[:n.value], dists[:n.value]


def t1_encode_cblk(coef, orient):
    a = np.ascontiguousarray(coef, dtype=np.int32)
    h, w = a.shape
    cap = w * h * 8 + 256
    out = np.empty(cap, np.uint8)
    nbps, npass = ctypes.c_uint32(), ctypes.c_uint32()
    rates = np.zeros(256, np.uint32)
    lens = np.zeros(256, np.uint32)
    n = lib().orc_t1_encode_cblk(a.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), w, h, w, orient, out.ctypes.data,
                                 cap, ctypes.byref(nbps), ctypes.byref(npass), rates.ctypes.data, lens.ctypes.data)
    return out[:n].tobytes(), nbps.value, npass.value, rates[:npass.value].copy(), lens[:npass.value].copy()


def t1_decode_cblk(data, npasses, numbps, orient, w, h):
    buf = np.frombuffer(data + b"\0" * 8, dtype=np.uint8).copy()
    out = np.empty((h, w), np.int32)
    lib().orc_t1_decode_cblk(buf.ctypes.data, len(data), npasses, numbps, orient, w, h,
                             out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)))
    return out


def ht_encode_cblk(coef):
    """HTJ2K cleanup-pass encode of one code-block of signed coefficients -> bytes."""
    a = np.ascontiguousarray(coef, dtype=np.int32)
    h, w = a.shape
    cap = w * h * 8 + 256
    out = np.empty(cap, np.uint8)
    n = lib().orc_ht_encode_cblk(a.ctypes.data, w, h, w, out.ctypes.data, cap)
    assert n >= 0
    return out[:n].tobytes()


def ht_decode_cblk(data, w, h, k_msbs=30):
    buf = np.frombuffer(data + b"\0" * 8, dtype=np.uint8).copy()
    out = np.empty((h, w), np.int32)
    rc = lib().orc_ht_decode_cblk(buf.ctypes.data, len(data), w, h, k_msbs, out.ctypes.data)
    if rc != 0:
        raise ValueError("HT block decode failed")
    return out


# ---------------------------------------------------------------- PNM helpers
def read_pnm(path):
    with open(path, "rb") as f:
        d = f.read()
    toks, i = [], 0
    while len(toks) < 4:
        while d[i:i + 1].isspace():
            i += 1
        if d[i:i + 1] == b"#":
            while d[i:i + 1] != b"\n":
                i += 1
            continue
        j = i
        while not d[j:j + 1].isspace():
            j += 1
        toks.append(d[i:j])
        i = j
    i += 1
    w, h, m = int(toks[1]), int(toks[2]), int(toks[3])
    c = 3 if toks[0] == b"P6" else 1
    dt = np.dtype(np.uint8) if m < 256 else np.dtype(">u2")
    a = np.frombuffer(d[i:i + w * h * c * dt.itemsize], dtype=dt).reshape(h, w, c)
    return np.ascontiguousarray(a.transpose(2, 0, 1)).astype(np.int32), m
