"""grok_amd — MI355X-native JPEG 2000 tile pipeline (host-side Python mirror).

The product is the C-ABI library ``libgrok_amd.so`` (include/grok_amd.h):
HIP kernels for gfx950 plus the native host engine (T2, codestream).  This
module binds it with ctypes and mirrors the reference's compress/decompress
call shape (grk_compress_* / grk_decompress_*, grok.h:1261-1451) for tests
and the benchmark.  There is no CPU fallback: if the extension cannot be
loaded, or no GPU is present, calls raise.
"""
import ctypes
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
# GROK_AMD_LIB: another in-tree build of the library (A/B measurements of kernel variants)
LIB_PATH = os.environ.get("GROK_AMD_LIB") or os.path.join(HERE, "libgrok_amd.so")

GK_MAXRLVLS = 33
GK_MAX_LAYERS = 100

# Exported symbols declared in include/grok_amd.h (checked by tests/test_capi.py).
EXPORTS = ("gk_create", "gk_destroy", "gk_set_default_params", "gk_encode", "gk_encode_tiles", "gk_main_header",
           "gk_jp2_header", "gk_decode_header", "gk_probe_header", "gk_decode", "gk_decode_window", "gk_get_timings",
           "gk_last_error", "gk_version", "gk_set_decode_layers", "gk_set_decode_reduce",
           "gk_set_window_rule", "gk_set_subsampling", "gk_probe_components", "gk_header_components")


class Poc(ctypes.Structure):
    """gk_poc (include/grok_amd.h): one progression order change."""
    _fields_ = [("resS", ctypes.c_uint32), ("compS", ctypes.c_uint32), ("layE", ctypes.c_uint32),
                ("resE", ctypes.c_uint32), ("compE", ctypes.c_uint32), ("prog", ctypes.c_int32)]


class CParameters(ctypes.Structure):
    """gk_cparameters (include/grok_amd.h) — subset of grk_cparameters (grok.h:466-590)."""
    _fields_ = [
        ("numlayers", ctypes.c_uint16),
        ("layer_rate", ctypes.c_double * GK_MAX_LAYERS),
        ("numresolution", ctypes.c_uint8),
        ("cblockw_init", ctypes.c_uint32), ("cblockh_init", ctypes.c_uint32),
        ("cblk_sty", ctypes.c_uint8), ("irreversible", ctypes.c_uint8), ("mct", ctypes.c_uint8),
        ("numgbits", ctypes.c_uint8), ("csty", ctypes.c_uint8),
        ("res_spec", ctypes.c_uint32),
        ("prcw_init", ctypes.c_uint32 * GK_MAXRLVLS), ("prch_init", ctypes.c_uint32 * GK_MAXRLVLS),
        ("write_comment", ctypes.c_uint8),
        ("tile_size_on", ctypes.c_uint8),
        ("t_width", ctypes.c_uint32), ("t_height", ctypes.c_uint32),
        ("writeTLM", ctypes.c_uint8), ("writePLT", ctypes.c_uint8),
        ("cod_format", ctypes.c_int32), ("prog_order", ctypes.c_int32),
        ("enableTilePartGeneration", ctypes.c_uint8), ("newTilePartProgressionDivider", ctypes.c_char),
        ("roi_compno", ctypes.c_int32), ("roi_shift", ctypes.c_uint32),
        ("numpocs", ctypes.c_uint32), ("pocs", Poc * 32),
        ("allocationByQuality", ctypes.c_uint8), ("layer_distortion", ctypes.c_double * GK_MAX_LAYERS),
        ("tx0", ctypes.c_uint32), ("ty0", ctypes.c_uint32),
        ("num_comments", ctypes.c_uint32), ("comment", ctypes.c_char_p * 256), ("comment_len", ctypes.c_uint16 * 256),
        ("is_binary_comment", ctypes.c_uint8 * 256),
    ]


class ImageInfo(ctypes.Structure):
    """gk_image_info; sample_bytes: 0/4 = int32 planes, 1/2 = planar 8/16-bit samples."""
    _fields_ = [(n, ctypes.c_uint32) for n in ("w", "h", "numcomps", "prec", "sgnd", "sample_bytes", "x0", "y0")]


class Timings(ctypes.Structure):
    _fields_ = [(n, ctypes.c_float) for n in ("mct_ms", "dwt_ms", "t1_ms", "t2_ms", "assemble_ms", "total_ms",
                                              "t1_cm_ms", "t1_coder_ms")] + \
               [("dwt_launches", ctypes.c_uint32), ("t1_blocks", ctypes.c_uint32)] + \
               [(n, ctypes.c_uint64) for n in ("dwt_bytes", "cs_bytes", "t1_bytes", "t1_steps_max", "t1_steps_total",
                                               "t1_symbols", "t1_solo_blocks", "t1_solo_decisions",
                                               "t1_solo_decisions_max")]


_lib = None


def load_library(build_if_missing=True):
    """Load the in-tree HIP extension (built by grok_amd.build / __graft_entry__.build)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        if not build_if_missing:
            raise RuntimeError("libgrok_amd.so is missing: run __graft_entry__.build()")
        from . import build as _b
        _b.build()
    lib = ctypes.CDLL(LIB_PATH)
    P = ctypes.POINTER
    lib.gk_create.restype = ctypes.c_void_p
    lib.gk_create.argtypes = [ctypes.c_int]
    lib.gk_destroy.argtypes = [ctypes.c_void_p]
    lib.gk_set_default_params.argtypes = [P(CParameters)]
    lib.gk_encode.restype = ctypes.c_int
    lib.gk_encode.argtypes = [ctypes.c_void_p, P(ImageInfo), P(ctypes.c_void_p), P(ctypes.c_uint32), ctypes.c_int,
                              P(CParameters), ctypes.c_void_p, ctypes.c_size_t, P(ctypes.c_size_t), ctypes.c_int]
    lib.gk_encode_tiles.restype = ctypes.c_int
    lib.gk_encode_tiles.argtypes = [ctypes.c_void_p, P(ImageInfo), P(ctypes.c_void_p), P(ctypes.c_uint32), ctypes.c_int,
                                    P(CParameters), ctypes.c_uint32, ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t,
                                    P(ctypes.c_size_t), P(ctypes.c_uint32), ctypes.c_int]
    lib.gk_main_header.restype = ctypes.c_int
    lib.gk_main_header.argtypes = [ctypes.c_void_p, P(ImageInfo), P(CParameters), ctypes.c_void_p, ctypes.c_size_t,
                                   P(ctypes.c_size_t), P(ctypes.c_size_t), P(ctypes.c_uint32)]
    lib.gk_jp2_header.restype = ctypes.c_int
    lib.gk_jp2_header.argtypes = [ctypes.c_void_p, P(ImageInfo), ctypes.c_uint64, ctypes.c_void_p, ctypes.c_size_t,
                                  P(ctypes.c_size_t)]
    lib.gk_probe_header.restype = ctypes.c_int
    lib.gk_probe_header.argtypes = [ctypes.c_void_p, ctypes.c_size_t, P(ImageInfo), P(CParameters), ctypes.c_char_p,
                                    ctypes.c_size_t]
    lib.gk_decode_window.restype = ctypes.c_int
    lib.gk_decode_window.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int] + \
        [ctypes.c_uint32] * 4 + [P(ctypes.c_void_p), P(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_int]
    lib.gk_decode_header.restype = ctypes.c_int
    lib.gk_decode_header.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, P(ImageInfo)]
    lib.gk_set_decode_reduce.restype = ctypes.c_int
    lib.gk_set_decode_reduce.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    lib.gk_set_window_rule.restype = ctypes.c_int
    lib.gk_set_window_rule.argtypes = [ctypes.c_void_p, ctypes.c_int]
    lib.gk_set_subsampling.restype = ctypes.c_int
    lib.gk_set_subsampling.argtypes = [ctypes.c_void_p, ctypes.c_uint32, P(ctypes.c_uint32), P(ctypes.c_uint32)]
    lib.gk_probe_components.restype = ctypes.c_int
    lib.gk_probe_components.argtypes = [ctypes.c_void_p, ctypes.c_size_t] + [P(ctypes.c_uint32)] * 4 + [ctypes.c_uint32]
    lib.gk_header_components.restype = ctypes.c_int
    lib.gk_header_components.argtypes = [ctypes.c_void_p] + [P(ctypes.c_uint32)] * 4 + [ctypes.c_uint32]
    lib.gk_set_decode_layers.restype = ctypes.c_int
    lib.gk_set_decode_layers.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    lib.gk_decode.restype = ctypes.c_int
    lib.gk_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int, P(ctypes.c_void_p),
                              P(ctypes.c_uint32), ctypes.c_uint32, ctypes.c_int]
    lib.gk_get_timings.restype = ctypes.c_int
    lib.gk_get_timings.argtypes = [ctypes.c_void_p, P(Timings)]
    lib.gk_last_error.restype = ctypes.c_char_p
    lib.gk_last_error.argtypes = [ctypes.c_void_p]
    lib.gk_version.restype = ctypes.c_char_p
    _lib = lib
    return lib


PROG_ORDERS = ["LRCP", "RLCP", "RPCL", "PCRL", "CPRL"]   # GRK_PROG_ORDER (grok.h)


def default_params(numresolution=6, cblk=(64, 64), irreversible=False, mct=True, numlayers=1, layer_rate=None,
                   precincts=None, write_comment=True, cblk_sty=0, tiles=None, tlm=False, plt=False, jp2=False,
                   prog_order="LRCP", tile_parts=None, pocs=None, roi=None, sop=False, eph=False, quality=None,
                   tile_origin=None, comments=None):
    """grk_compress_set_default_params + the CLI options used by the benchmark configs.

    prog_order: "LRCP", "RLCP", "RPCL", "PCRL", "CPRL" or 0..4 (grk_compress -p).
    cblk_sty=0x40 selects the HTJ2K block coder; like grk_compress -M 64
    (grk_compress.cpp:1120-1125) it also sets one guard bit."""
    lib = load_library()
    p = CParameters()
    lib.gk_set_default_params(ctypes.byref(p))
    p.numresolution = numresolution
    if tile_origin:   # grk_compress -T: the tile grid's canvas origin (the image origin is Engine.encode's `origin`)
        p.tx0, p.ty0 = int(tile_origin[0]), int(tile_origin[1])
    p.cblockw_init, p.cblockh_init = cblk
    p.irreversible = int(irreversible)
    p.mct = int(mct)
    p.numlayers = len(layer_rate) if layer_rate else numlayers
    if layer_rate:
        for i, r in enumerate(layer_rate):
            p.layer_rate[i] = r
    if precincts:
        p.csty |= 1
        p.res_spec = len(precincts)
        for i, (w, h) in enumerate(precincts):
            p.prcw_init[i], p.prch_init[i] = w, h
    p.write_comment = int(write_comment)
    p.cblk_sty = int(cblk_sty)
    if cblk_sty & 0x40:
        p.numgbits = 1
    if tiles:   # grk_compress -t W,H
        p.tile_size_on = 1
        p.t_width, p.t_height = int(tiles[0]), int(tiles[1])
    p.writeTLM, p.writePLT = int(bool(tlm)), int(bool(plt))
    p.cod_format = 2 if jp2 else 0   # GRK_CODEC_JP2 / GRK_CODEC_J2K
    p.prog_order = PROG_ORDERS.index(prog_order) if isinstance(prog_order, str) else int(prog_order)
    p.roi_compno, p.roi_shift = (int(roi[0]), int(roi[1])) if roi else (-1, 0)   # grk_compress -ROI c=..,U=..
    if pocs:   # [(resS, compS, layE, resE, compE, "PROG"), ...] (grk_compress -P)
        p.numpocs = len(pocs)
        for i, (rs, cs, le, re_, ce, pr) in enumerate(pocs):
            p.pocs[i] = Poc(rs, cs, le, re_, ce, PROG_ORDERS.index(pr) if isinstance(pr, str) else int(pr))
    if tile_parts:   # grk_compress -u L|R|C: a new tile part whenever that index changes
        p.enableTilePartGeneration = 1
        p.newTilePartProgressionDivider = tile_parts.encode()
    p.csty |= (2 if sop else 0) | (4 if eph else 0)   # grk_compress -S / -E
    if comments:   # grk_compress -C: [bytes or str, ...] (bytes = binary, Rcom 0); the buffers stay with p
        p._comment_bufs = [c if isinstance(c, bytes) else c.encode() for c in comments]
        p.num_comments = len(comments)
        for i, c in enumerate(comments):
            p.comment[i] = p._comment_bufs[i]
            p.comment_len[i] = len(p._comment_bufs[i])
            p.is_binary_comment[i] = 1 if isinstance(c, bytes) else 0
    if quality:   # grk_compress -q PSNR,PSNR,...: fixed-quality layers
        p.allocationByQuality = 1
        p.numlayers = len(quality)
        for i, q in enumerate(quality):
            p.layer_distortion[i] = q
    return p


def probe_header(cs):
    """gk_probe_header: image info of host codestream / JP2 bytes, no engine or GPU needed."""
    lib = load_library()
    b = np.frombuffer(bytes(cs), np.uint8)
    info = ImageInfo()
    msg = ctypes.create_string_buffer(256)
    if lib.gk_probe_header(b.ctypes.data, len(b), ctypes.byref(info), None, msg, 256) != 0:
        raise ValueError(msg.value.decode())
    return info


def probe_components(cs, precision=False):
    """gk_probe_components: [(dx, dy)] per component of host codestream / JP2 bytes (SIZ XRsiz /
    YRsiz); with precision=True [(dx, dy, prec, signed)]."""
    lib = load_library()
    b = np.frombuffer(bytes(cs), np.uint8)
    dx, dy, pr, sg = [(ctypes.c_uint32 * 16384)() for _ in range(4)]
    n = lib.gk_probe_components(b.ctypes.data, len(b), dx, dy, pr, sg, 16384)
    if n < 0:
        raise ValueError("gk_probe_components failed")
    if precision:
        return [(dx[c], dy[c], pr[c], bool(sg[c])) for c in range(n)]
    return [(dx[c], dy[c]) for c in range(n)]


def comp_shape(w, h, dx, dy, origin=(0, 0), reduce=0):
    """(rows, cols) of a component sampled every (dx, dy) canvas positions over the image area
    [x0, x0 + w) x [y0, y0 + h) (grk_image_comp h / w), reduced by `reduce` resolutions."""
    x0, y0 = origin
    cd = lambda a, b: -(-a // b)
    cx0, cy0, cx1, cy1 = cd(x0, dx), cd(y0, dy), cd(x0 + w, dx), cd(y0 + h, dy)
    r = 1 << reduce
    return cd(cy1, r) - cd(cy0, r), cd(cx1, r) - cd(cx0, r)


def _sample_bytes(x):
    """gk_image_info::sample_bytes of a plane array (numpy or torch): 0 for 32-bit, else its item size."""
    n = x.element_size() if hasattr(x, "element_size") else x.dtype.itemsize
    return 0 if n == 4 else n


def _host_planes(a, prec):
    """Host planes as passed when their 8/16-bit type fits the precision ((prec + 7) // 8 bytes,
    grk_compress_tile's raw buffer), int32 otherwise."""
    if a.dtype.kind in "ui" and a.dtype.itemsize in (1, 2) and a.dtype.itemsize == (prec + 7) // 8:
        return np.ascontiguousarray(a)
    return np.ascontiguousarray(a, dtype=np.int32)


def _np_sample_dtype(sample_bytes, info):
    if sample_bytes in (0, 4):
        return np.int32
    return {(1, 0): np.uint8, (1, 1): np.int8, (2, 0): np.uint16, (2, 1): np.int16}[(sample_bytes, int(info.sgnd))]


def _is_torch_cuda(x):
    return hasattr(x, "is_cuda") and x.is_cuda


class Engine:
    """One MI355X, one HIP stream (grk_codec analogue)."""

    def __init__(self, device=0):
        # PyTorch-ROCm bundles its own HIP/HSA runtime.  When both live in one
        # process, torch's must initialise first or it later reports "No HIP
        # GPUs"; device tensors are only exchanged with torch, so initialise it
        # here when it is present.  The C ABI itself does not depend on torch.
        if "torch" in sys.modules:
            try:
                sys.modules["torch"].cuda.init()
            except Exception:
                pass
        self.lib = load_library()
        self.ctx = self.lib.gk_create(device)
        if not self.ctx:
            raise RuntimeError("gk_create failed: no HIP device %d" % device)

    def close(self):
        if self.ctx:
            self.lib.gk_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _err(self, what):
        raise RuntimeError("%s failed: %s" % (what, self.lib.gk_last_error(self.ctx).decode()))

    def timings(self):
        t = Timings()
        self.lib.gk_get_timings(self.ctx, ctypes.byref(t))
        return t

    # ------------------------------------------------------------------ encode
    def encode(self, planes, prec, signed=False, params=None, out=None, origin=None, subsampling=None, size=None):
        """planes: (C, H, W) int32 numpy array (host) or torch cuda tensor (device).
        Returns bytes (host) or, when ``out`` (a torch cuda uint8 tensor) is given,
        the codestream length written into it on the device.  origin: the image area's
        canvas origin (grk_image::x0 / y0, grk_compress -d); without it the image sits at
        the tile grid origin (-T alone moves the image there, grk_compress.cpp:1547-1551).
        subsampling=[(dx, dy), ...] (grk_image_comp::dx / dy): planes is then a list of 2-D
        planes of comp_shape(W, H, dx, dy, origin) each and size=(W, H) the image area."""
        if params is None:
            params = default_params()
        if subsampling:
            return self._encode_subsampled(planes, prec, signed, params, out, origin, subsampling, size)
        c, h, w = planes.shape
        on_dev = _is_torch_cuda(planes)
        if on_dev:
            assert planes.is_contiguous() and planes.element_size() in (1, 2, 4)
            base = planes.data_ptr()
        else:
            planes = _host_planes(planes, prec)
            base = planes.ctypes.data
        sb = _sample_bytes(planes)
        es = sb or 4
        info = ImageInfo(w, h, c, prec, int(signed), sb)
        if origin is not None:
            info.x0, info.y0 = int(origin[0]), int(origin[1])
        else:
            info.x0, info.y0 = params.tx0, params.ty0
        ptrs = (ctypes.c_void_p * c)(*[base + k * h * w * es for k in range(c)])
        strides = (ctypes.c_uint32 * c)(*([w] * c))
        n = ctypes.c_size_t()
        if out is not None:
            rc = self.lib.gk_encode(self.ctx, ctypes.byref(info), ptrs, strides, int(on_dev), ctypes.byref(params),
                                    ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(n), 1)
            if rc != 0:
                self._err("gk_encode")
            return n.value
        cap = c * h * w * 4 + (1 << 20)
        buf = np.empty(cap, np.uint8)
        rc = self.lib.gk_encode(self.ctx, ctypes.byref(info), ptrs, strides, int(on_dev), ctypes.byref(params),
                                buf.ctypes.data, cap, ctypes.byref(n), 0)
        if rc == -2:
            buf = np.empty(n.value, np.uint8)
            rc = self.lib.gk_encode(self.ctx, ctypes.byref(info), ptrs, strides, int(on_dev), ctypes.byref(params),
                                    buf.ctypes.data, n.value, ctypes.byref(n), 0)
        if rc != 0:
            self._err("gk_encode")
        return buf[:n.value].tobytes()

    def _encode_subsampled(self, planes, prec, signed, params, out, origin, subsampling, size):
        c = len(planes)
        w, h = size
        on_dev = _is_torch_cuda(planes[0])
        keep = [p if on_dev else _host_planes(p, prec) for p in planes]
        sb = _sample_bytes(keep[0])
        info = ImageInfo(w, h, c, prec, int(signed), sb)
        if origin is not None:
            info.x0, info.y0 = int(origin[0]), int(origin[1])
        else:
            info.x0, info.y0 = params.tx0, params.ty0
        for k, (dx, dy) in enumerate(subsampling):
            assert tuple(keep[k].shape) == comp_shape(w, h, dx, dy, (info.x0, info.y0)), (k, tuple(keep[k].shape))
        ptrs = (ctypes.c_void_p * c)(*[p.data_ptr() if on_dev else p.ctypes.data for p in keep])
        strides = (ctypes.c_uint32 * c)(*[p.shape[1] for p in keep])
        dxs = (ctypes.c_uint32 * c)(*[int(d[0]) for d in subsampling])
        dys = (ctypes.c_uint32 * c)(*[int(d[1]) for d in subsampling])
        if self.lib.gk_set_subsampling(self.ctx, c, dxs, dys) != 0:
            self._err("gk_set_subsampling")
        try:
            n = ctypes.c_size_t()
            if out is not None:
                rc = self.lib.gk_encode(self.ctx, ctypes.byref(info), ptrs, strides, int(on_dev), ctypes.byref(params),
                                        ctypes.c_void_p(out.data_ptr()), out.numel(), ctypes.byref(n), 1)
                if rc != 0:
                    self._err("gk_encode")
                return n.value
            cap = c * h * w * 4 + (1 << 20)
            buf = np.empty(cap, np.uint8)
            rc = self.lib.gk_encode(self.ctx, ctypes.byref(info), ptrs, strides, int(on_dev), ctypes.byref(params),
                                    buf.ctypes.data, cap, ctypes.byref(n), 0)
            if rc != 0:
                self._err("gk_encode")
            return buf[:n.value].tobytes()
        finally:
            self.lib.gk_set_subsampling(self.ctx, 0, None, None)

    def encode_tiles_subsampled(self, planes, prec, tile_begin, tile_end, subsampling, size, signed=False, params=None,
                                origin=None):
        """gk_encode_tiles for an image with subsampled components: planes = whole component
        planes (comp_shape each); only the rows of the selected tiles are read.  Returns
        (bytes, part_lens); with main_header_subsampled and EOC the parts assemble the stream."""
        if params is None:
            params = default_params()
        c = len(planes)
        w, h = size
        keep = [_host_planes(p, prec) for p in planes]
        info = ImageInfo(w, h, c, prec, int(signed), _sample_bytes(keep[0]))
        info.x0, info.y0 = (int(origin[0]), int(origin[1])) if origin is not None else (params.tx0, params.ty0)
        ptrs = (ctypes.c_void_p * c)(*[p.ctypes.data for p in keep])
        strides = (ctypes.c_uint32 * c)(*[p.shape[1] for p in keep])
        dxs = (ctypes.c_uint32 * c)(*[int(d[0]) for d in subsampling])
        dys = (ctypes.c_uint32 * c)(*[int(d[1]) for d in subsampling])
        if self.lib.gk_set_subsampling(self.ctx, c, dxs, dys) != 0:
            self._err("gk_set_subsampling")
        try:
            lens = (ctypes.c_uint32 * (tile_end - tile_begin))()
            n = ctypes.c_size_t()
            cap = sum(p.size for p in keep) * 4 + (1 << 20)
            buf = np.empty(cap, np.uint8)
            rc = self.lib.gk_encode_tiles(self.ctx, ctypes.byref(info), ptrs, strides, 0, ctypes.byref(params),
                                          tile_begin, tile_end, buf.ctypes.data, cap, ctypes.byref(n), lens, 0)
            if rc != 0:
                self._err("gk_encode_tiles")
            hdr = np.empty(1 << 20, np.uint8)
            hn, tlm, nt = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_uint32()
            if self.lib.gk_main_header(self.ctx, ctypes.byref(info), ctypes.byref(params), hdr.ctypes.data, hdr.size,
                                       ctypes.byref(hn), ctypes.byref(tlm), ctypes.byref(nt)) != 0:
                self._err("gk_main_header")
            return hdr[:hn.value].tobytes(), buf[:n.value].tobytes(), list(lens)
        finally:
            self.lib.gk_set_subsampling(self.ctx, 0, None, None)

    def subsampling(self):
        """[(dx, dy)] per component of the stream the last read_header / decode read."""
        dx, dy = (ctypes.c_uint32 * 16384)(), (ctypes.c_uint32 * 16384)()
        n = self.lib.gk_header_components(self.ctx, dx, dy, None, None, 16384)
        return [(dx[c], dy[c]) for c in range(max(n, 0))]

    def _planes_ptrs(self, planes, row0=0, prec=32):
        """Component base pointers addressing image row 0 for a (C, rows, W) slab whose
        first row is image row ``row0`` (only the slab's rows are ever read)."""
        c, h, w = planes.shape
        if _is_torch_cuda(planes):
            assert planes.is_contiguous() and planes.element_size() in (1, 2, 4)
            base, keep = planes.data_ptr(), planes
        else:
            keep = _host_planes(planes, prec)
            base = keep.ctypes.data
        es = _sample_bytes(keep) or 4
        ptrs = (ctypes.c_void_p * c)(*[base + k * h * w * es - row0 * w * es for k in range(c)])
        return ptrs, keep

    def encode_tiles(self, planes, prec, tile_begin, tile_end, image_hw=None, row0=0, signed=False, params=None,
                     out=None):
        """gk_encode_tiles: tile parts of tiles [tile_begin, tile_end) only (tile sharding).
        planes: (C, rows, W) slab starting at image row ``row0`` (the whole image by
        default); image_hw = (H, W) of the full image.  Returns (bytes or length, part_lens)."""
        if params is None:
            params = default_params()
        c, h, w = planes.shape
        H, W = image_hw if image_hw else (h, w)
        assert W == w
        ptrs, keep = self._planes_ptrs(planes, row0, prec)
        info = ImageInfo(W, H, c, prec, int(signed), _sample_bytes(keep))
        info.x0, info.y0 = params.tx0, params.ty0
        on_dev = _is_torch_cuda(planes)
        strides = (ctypes.c_uint32 * c)(*([w] * c))
        lens = (ctypes.c_uint32 * (tile_end - tile_begin))()
        n = ctypes.c_size_t()
        if out is not None:
            rc = self.lib.gk_encode_tiles(self.ctx, ctypes.byref(info), ptrs, strides, int(on_dev), ctypes.byref(params),
                                          tile_begin, tile_end, ctypes.c_void_p(out.data_ptr()), out.numel(),
                                          ctypes.byref(n), lens, 1)
            if rc != 0:
                self._err("gk_encode_tiles")
            return n.value, list(lens)
        cap = c * h * w * 4 + (1 << 20)
        buf = np.empty(cap, np.uint8)
        rc = self.lib.gk_encode_tiles(self.ctx, ctypes.byref(info), ptrs, strides, int(on_dev), ctypes.byref(params),
                                      tile_begin, tile_end, buf.ctypes.data, cap, ctypes.byref(n), lens, 0)
        if rc != 0:
            self._err("gk_encode_tiles")
        del keep
        return buf[:n.value].tobytes(), list(lens)

    def jp2_header(self, image_shape, prec, cs_len, signed=False):
        """gk_jp2_header: the JP2 boxes in front of a codestream of cs_len bytes."""
        c, h, w = image_shape
        info = ImageInfo(w, h, c, prec, int(signed), 0)
        buf = np.empty(256, np.uint8)
        n = ctypes.c_size_t()
        if self.lib.gk_jp2_header(self.ctx, ctypes.byref(info), cs_len, buf.ctypes.data, buf.size, ctypes.byref(n)) != 0:
            self._err("gk_jp2_header")
        return buf[:n.value].tobytes()

    def main_header(self, image_shape, prec, signed=False, params=None):
        """gk_main_header: (header bytes, TLM entry offset or 0, number of tiles)."""
        if params is None:
            params = default_params()
        c, h, w = image_shape
        info = ImageInfo(w, h, c, prec, int(signed), 0)
        info.x0, info.y0 = params.tx0, params.ty0
        buf = np.empty(1 << 20, np.uint8)
        n, tlm, nt = ctypes.c_size_t(), ctypes.c_size_t(), ctypes.c_uint32()
        rc = self.lib.gk_main_header(self.ctx, ctypes.byref(info), ctypes.byref(params), buf.ctypes.data, buf.size,
                                     ctypes.byref(n), ctypes.byref(tlm), ctypes.byref(nt))
        if rc != 0:
            self._err("gk_main_header")
        return buf[:n.value].tobytes(), tlm.value, nt.value

    # ------------------------------------------------------------------ decode
    def read_header(self, cs, length=None):
        info = ImageInfo()
        if _is_torch_cuda(cs):
            rc = self.lib.gk_decode_header(self.ctx, ctypes.c_void_p(cs.data_ptr()), length, 1, ctypes.byref(info))
        else:
            b = np.frombuffer(cs, np.uint8)
            rc = self.lib.gk_decode_header(self.ctx, b.ctypes.data, len(cs), 0, ctypes.byref(info))
        if rc != 0:
            self._err("gk_decode_header")
        return info

    def decode_window(self, cs, window, length=None, out=None, sample_bytes=0):
        """gk_decode_window: window = (x0, y0, x1, y1).  Returns a (C, y1-y0, x1-x0) numpy
        array (int32, or 8/16-bit with sample_bytes 1/2), or fills ``out`` (a torch cuda
        tensor of that shape; its element size selects the sample type) in place.  With
        set_decode_reduce(r) the window (full-resolution coordinates) is returned at the
        reduced resolution: its canvas rectangle with every edge ceil(x / 2^r)."""
        on_dev = _is_torch_cuda(cs)
        info = self.read_header(cs, length)
        x0, y0, x1, y1 = window
        c, h, w = info.numcomps, y1 - y0, x1 - x0
        sub = self.subsampling()
        if any(d != (1, 1) for d in sub):
            return self._window_subsampled(cs, length, window, out, sample_bytes, info, sub)
        red = getattr(self, "_reduce", 0)
        if red:   # the window's canvas rectangle reduced: ceil(x / 2^reduce) (set_decode_reduce)
            cd = lambda v: -(-v >> red)
            w = cd(x1 + info.x0) - cd(x0 + info.x0)
            h = cd(y1 + info.y0) - cd(y0 + info.y0)
        if out is not None:
            # any (C, h, w) view with unit column stride (e.g. a row band of a larger window)
            assert tuple(out.shape) == (c, h, w) and out.stride(2) == 1
            base, res, out_dev = out.data_ptr(), out, 1
            sample_bytes = _sample_bytes(out)
            es = sample_bytes or 4
            cstride, rstride = out.stride(0), out.stride(1)
        else:
            res = np.empty((c, h, w), _np_sample_dtype(sample_bytes, info))
            base, out_dev = res.ctypes.data, 0
            es = sample_bytes or 4
            cstride, rstride = h * w, w
        strides = (ctypes.c_uint32 * c)(*([rstride] * c))
        ptrs = (ctypes.c_void_p * c)(*[base + k * cstride * es for k in range(c)])
        if on_dev:
            rc = self.lib.gk_decode_window(self.ctx, ctypes.c_void_p(cs.data_ptr()), length, 1, x0, y0, x1, y1, ptrs,
                                           strides, sample_bytes, out_dev)
        else:
            b = np.frombuffer(cs, np.uint8)
            rc = self.lib.gk_decode_window(self.ctx, b.ctypes.data, len(cs), 0, x0, y0, x1, y1, ptrs, strides,
                                           sample_bytes, out_dev)
        if rc != 0:
            self._err("gk_decode_window")
        return res

    def set_decode_layers(self, max_layers):
        """gk_set_decode_layers: decode only the first max_layers quality layers (0 = all),
        as grk_decompress -l (grk_dparameters::cp_layer)."""
        if self.lib.gk_set_decode_layers(self.ctx, int(max_layers)) != 0:
            self._err("gk_set_decode_layers")

    def set_decode_reduce(self, reduce):
        """gk_set_decode_reduce: discard the `reduce` highest resolutions (grk_decompress -r,
        grk_dparameters::cp_reduce); decode() then returns ceil(H / 2^reduce) x ceil(W / 2^reduce)."""
        if self.lib.gk_set_decode_reduce(self.ctx, int(reduce)) != 0:
            self._err("gk_set_decode_reduce")
        self._reduce = int(reduce)

    def set_window_rule(self, whole_tile):
        """gk_set_window_rule: later windows use Grok's whole-tile inverse 5/3 rule (True, as
        decompressTile without a window) or its partial-tile rule (False, the default)."""
        if self.lib.gk_set_window_rule(self.ctx, int(bool(whole_tile))) != 0:
            self._err("gk_set_window_rule")

    def decode(self, cs, length=None, out=None, row0=0, sample_bytes=0):
        """cs: bytes (host) or torch cuda uint8 tensor (+length).  Returns a (C, H, W)
        numpy array (int32, or 8/16-bit with sample_bytes 1/2), or fills ``out`` (torch
        cuda tensor; its element size selects the sample type) in place.  ``out`` may be
        a (C, rows, W) slab holding image rows [row0, row0+rows) when cs carries only the
        tile parts of those rows (sharded decode)."""
        on_dev = _is_torch_cuda(cs)
        info = self.read_header(cs, length)
        c, h, w = info.numcomps, info.h, info.w
        red = getattr(self, "_reduce", 0)
        sub = self.subsampling()
        if any(d != (1, 1) for d in sub):
            return self._decode_subsampled(cs, length, out, sample_bytes, info, sub, red)
        if red:   # reduced-resolution output: the image area on the reduced canvas (ceil(x / 2^reduce))
            cd = lambda v: -(-v // (1 << red))
            h, w = cd(info.y0 + h) - cd(info.y0), cd(info.x0 + w) - cd(info.x0)
        strides = (ctypes.c_uint32 * c)(*([w] * c))
        if out is not None:
            sample_bytes = _sample_bytes(out)
            es = sample_bytes or 4
            base = out.data_ptr()
            rows = out.shape[1]
            ptrs = (ctypes.c_void_p * c)(*[base + k * rows * w * es - row0 * w * es for k in range(c)])
            res, out_dev = out, 1
        else:
            es = sample_bytes or 4
            res = np.empty((c, h, w), _np_sample_dtype(sample_bytes, info))
            base = res.ctypes.data
            ptrs = (ctypes.c_void_p * c)(*[base + k * h * w * es for k in range(c)])
            out_dev = 0
        if on_dev:
            rc = self.lib.gk_decode(self.ctx, ctypes.c_void_p(cs.data_ptr()), length, 1, ptrs, strides, sample_bytes,
                                    out_dev)
        else:
            b = np.frombuffer(cs, np.uint8)
            rc = self.lib.gk_decode(self.ctx, b.ctypes.data, len(cs), 0, ptrs, strides, sample_bytes, out_dev)
        if rc != 0:
            self._err("gk_decode")
        return res

    def _decode_subsampled(self, cs, length, out, sample_bytes, info, sub, red):
        """Subsampled components: a list of 2-D planes, component c of comp_shape(W, H, dx, dy,
        origin, reduce); ``out`` (torch cuda) is then a list of such tensors filled in place."""
        c = info.numcomps
        shapes = [comp_shape(info.w, info.h, dx, dy, (info.x0, info.y0), red) for dx, dy in sub]
        if out is not None:
            assert len(out) == c and all(tuple(o.shape) == s for o, s in zip(out, shapes))
            sample_bytes = _sample_bytes(out[0])
            res, out_dev = out, 1
            ptrs = (ctypes.c_void_p * c)(*[o.data_ptr() for o in out])
            strides = (ctypes.c_uint32 * c)(*[o.stride(0) for o in out])
        else:
            res = [np.empty(s, _np_sample_dtype(sample_bytes, info)) for s in shapes]
            out_dev = 0
            ptrs = (ctypes.c_void_p * c)(*[r.ctypes.data for r in res])
            strides = (ctypes.c_uint32 * c)(*[s[1] for s in shapes])
        if _is_torch_cuda(cs):
            rc = self.lib.gk_decode(self.ctx, ctypes.c_void_p(cs.data_ptr()), length, 1, ptrs, strides, sample_bytes,
                                    out_dev)
        else:
            b = np.frombuffer(cs, np.uint8)
            rc = self.lib.gk_decode(self.ctx, b.ctypes.data, len(cs), 0, ptrs, strides, sample_bytes, out_dev)
        if rc != 0:
            self._err("gk_decode")
        return res

    def _window_subsampled(self, cs, length, window, out, sample_bytes, info, sub):
        """Window of a stream with subsampled components: component c's plane is the window's
        canvas rectangle on its grid (every edge ceil(x / dx), then reduced), a list of planes."""
        x0, y0, x1, y1 = window
        red = getattr(self, "_reduce", 0)
        cd = lambda a, b: -(-a // b)
        shapes = []
        for dx, dy in sub:
            gx = lambda v: cd(cd(v + info.x0, dx), 1 << red)
            gy = lambda v: cd(cd(v + info.y0, dy), 1 << red)
            shapes.append((gy(y1) - gy(y0), gx(x1) - gx(x0)))
        c = info.numcomps
        if out is not None:
            assert len(out) == c and all(tuple(o.shape) == s for o, s in zip(out, shapes))
            sample_bytes = _sample_bytes(out[0])
            res, out_dev = out, 1
            ptrs = (ctypes.c_void_p * c)(*[o.data_ptr() for o in out])
            strides = (ctypes.c_uint32 * c)(*[o.stride(0) for o in out])
        else:
            res = [np.empty(s, _np_sample_dtype(sample_bytes, info)) for s in shapes]
            out_dev = 0
            ptrs = (ctypes.c_void_p * c)(*[r.ctypes.data for r in res])
            strides = (ctypes.c_uint32 * c)(*[max(s[1], 1) for s in shapes])
        if _is_torch_cuda(cs):
            rc = self.lib.gk_decode_window(self.ctx, ctypes.c_void_p(cs.data_ptr()), length, 1, x0, y0, x1, y1, ptrs,
                                           strides, sample_bytes, out_dev)
        else:
            b = np.frombuffer(cs, np.uint8)
            rc = self.lib.gk_decode_window(self.ctx, b.ctypes.data, len(cs), 0, x0, y0, x1, y1, ptrs, strides,
                                           sample_bytes, out_dev)
        if rc != 0:
            self._err("gk_decode_window")
        return res
