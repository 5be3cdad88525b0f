"""OpenJPEG 2.5.4 (the libopenjp2 Pillow ships) driven through its C API with ctypes: an
independent decoder that returns every component at its own size.

Pillow's own JPEG 2000 plugin refuses subsampled components except as sYCC, which it converts to
RGB; the library itself decodes them plane by plane (opj_image_comp_t w / h / dx / dy), which is
what the subsampling tests compare against.  Test infrastructure only."""
import ctypes
import glob
import os
import tempfile

import numpy as np

_lib = None


def _find():
    try:
        import PIL
    except ImportError:
        return None
    d = os.path.join(os.path.dirname(os.path.dirname(PIL.__file__)), "pillow.libs")
    hits = sorted(glob.glob(os.path.join(d, "libopenjp2*.so*")))
    return hits[0] if hits else None


class _Comp(ctypes.Structure):   # opj_image_comp_t (openjpeg.h, 2.5)
    _fields_ = [("dx", ctypes.c_uint32), ("dy", ctypes.c_uint32), ("w", ctypes.c_uint32), ("h", ctypes.c_uint32),
                ("x0", ctypes.c_uint32), ("y0", ctypes.c_uint32), ("prec", ctypes.c_uint32), ("bpp", ctypes.c_uint32),
                ("sgnd", ctypes.c_uint32), ("resno_decoded", ctypes.c_uint32), ("factor", ctypes.c_uint32),
                ("data", ctypes.POINTER(ctypes.c_int32)), ("alpha", ctypes.c_uint16)]


class _Image(ctypes.Structure):  # opj_image_t
    _fields_ = [("x0", ctypes.c_uint32), ("y0", ctypes.c_uint32), ("x1", ctypes.c_uint32), ("y1", ctypes.c_uint32),
                ("numcomps", ctypes.c_uint32), ("color_space", ctypes.c_int), ("comps", ctypes.POINTER(_Comp)),
                ("icc_profile_buf", ctypes.c_void_p), ("icc_profile_len", ctypes.c_uint32)]


def available():
    return _find() is not None


def lib():
    global _lib
    if _lib is None:
        path = _find()
        if path is None:
            raise RuntimeError("libopenjp2 not found")
        L = ctypes.CDLL(path)
        L.opj_version.restype = ctypes.c_char_p
        L.opj_create_decompress.restype = ctypes.c_void_p
        L.opj_create_decompress.argtypes = [ctypes.c_int]
        L.opj_set_default_decoder_parameters.argtypes = [ctypes.c_void_p]
        L.opj_setup_decoder.restype = ctypes.c_int
        L.opj_setup_decoder.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.opj_stream_create_default_file_stream.restype = ctypes.c_void_p
        L.opj_stream_create_default_file_stream.argtypes = [ctypes.c_char_p, ctypes.c_int]
        L.opj_read_header.restype = ctypes.c_int
        L.opj_read_header.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.POINTER(_Image))]
        L.opj_decode.restype = ctypes.c_int
        L.opj_decode.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(_Image)]
        L.opj_end_decompress.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
        L.opj_stream_destroy.argtypes = [ctypes.c_void_p]
        L.opj_destroy_codec.argtypes = [ctypes.c_void_p]
        L.opj_image_destroy.argtypes = [ctypes.POINTER(_Image)]
        _lib = L
    return _lib


def version():
    return lib().opj_version().decode()


def decode(cs):
    """Decode a raw codestream (J2K) -> [(dx, dy, plane int32 (h, w))] per component."""
    L = lib()
    with tempfile.NamedTemporaryFile(suffix=".j2k", delete=False) as f:
        f.write(cs)
        path = f.name
    codec = stream = None
    img = ctypes.POINTER(_Image)()
    try:
        codec = L.opj_create_decompress(0)   # OPJ_CODEC_J2K
        params = ctypes.create_string_buffer(1 << 16)   # opj_dparameters_t (a few KB)
        L.opj_set_default_decoder_parameters(params)
        if not L.opj_setup_decoder(codec, params):
            raise RuntimeError("opj_setup_decoder failed")
        stream = L.opj_stream_create_default_file_stream(path.encode(), 1)
        if not stream or not L.opj_read_header(stream, codec, ctypes.byref(img)):
            raise RuntimeError("opj_read_header failed")
        if not L.opj_decode(codec, stream, img):
            raise RuntimeError("opj_decode failed")
        L.opj_end_decompress(codec, stream)
        out = []
        for c in range(img.contents.numcomps):
            cp = img.contents.comps[c]
            a = np.ctypeslib.as_array(cp.data, shape=(cp.h, cp.w)).copy()
            out.append((cp.dx, cp.dy, a))
        return out
    finally:
        if img:
            L.opj_image_destroy(img)
        if stream:
            L.opj_stream_destroy(stream)
        if codec:
            L.opj_destroy_codec(codec)
        os.unlink(path)
