"""B1 drop-in boundary without a GPU: include/grk_abi.h (the grk_* API served by
libgrok_amd.so) against the reference's public header.

* every struct a caller of Grok's C API touches has grok.h's size and the same offset
  for every field (both headers compiled by gcc; a program prints sizeof / offsetof);
* libgrok_amd.so exports every function grok.h declares (GRK_API), under its name;
* entry points that need no GPU behave like Grok's: default parameters, images,
  memory streams, reference counting, plugin calls reporting "not handled".

/root/reference is read as text here (the CPU suite only); the layout program compiles
grok.h's declarations with its generated-config include line dropped (it only defines
version macros).  Skipped when the reference is absent (the GPU box)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT
import grok_amd as G

REF_H = "/root/reference/src/lib/jp2/grok.h"
ABI_H = os.path.join(ROOT, "include", "grk_abi.h")


def _structs(path):
    """{typedef name: [field names]} of the struct typedefs in a header."""
    txt = re.sub(r"/\*.*?\*/", "", open(path).read(), flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    out = {}
    for m in re.finditer(r"typedef\s+struct\s*\w*\s*\{([^{}]*)\}\s*(\w+)\s*;", txt):
        body, name = m.group(1), m.group(2)
        fields = []
        for decl in body.split(";"):
            decl = " ".join(decl.split())
            if not decl:
                continue
            for k, part in enumerate(decl.split(",")):
                fm = re.search(r"(\w+)\s*(\[[^\]]*\])?\s*$", part.strip())
                fields.append(fm.group(1))
        out[name] = fields
    return out


def _layout(header_text, structs, tmp, tag):
    src = tmp / ("layout_%s.c" % tag)
    lines = [header_text, "#include <stddef.h>", "int main(void) {"]
    for s, fields in sorted(structs.items()):
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (s, s))
        for f in fields:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (s, f, s, f))
    lines.append("return 0; }")
    src.write_text("\n".join(lines))
    exe = tmp / ("layout_%s" % tag)
    subprocess.check_call(["gcc", "-std=c11", "-w", str(src), "-o", str(exe)])
    return subprocess.check_output([str(exe)]).decode().split("\n")


@pytest.mark.skipif(not os.path.exists(REF_H), reason="reference header not present")
def test_struct_layouts_match_reference(tmp_path):
    mine = _structs(ABI_H)
    ref = _structs(REF_H)
    shared = {k: v for k, v in mine.items() if k in ref}
    # every reference struct of the API surface is mirrored, with the same fields in the same order
    assert set(ref) <= set(mine), sorted(set(ref) - set(mine))
    for k in shared:
        assert mine[k] == ref[k], k
    ref_text = "\n".join(l for l in open(REF_H).read().split("\n") if '#include "grk_config.h"' not in l)
    got = _layout('#include "%s"' % ABI_H, shared, tmp_path, "abi")
    want = _layout(ref_text, shared, tmp_path, "ref")
    assert got == want


@pytest.mark.skipif(not os.path.exists(REF_H), reason="reference header not present")
def test_every_grok_entry_point_is_exported():
    txt = re.sub(r"/\*.*?\*/", "", open(REF_H).read(), flags=re.S)
    names = set(re.findall(r"GRK_API\s+[\w\s\*]+?GRK_CALLCONV\s+(grk_\w+)\s*\(", txt))
    assert len(names) >= 50
    out = subprocess.run(["nm", "-D", "--defined-only", G.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    assert not sorted(names - exported), sorted(names - exported)


def _lib():
    return G.load_library()


def test_compress_default_params_match_grok():
    # grk_compress_set_default_params (grok.cpp:405-435), read through the ctypes view of the ABI
    lib = _lib()
    buf = ctypes.create_string_buffer(1 << 20)
    lib.grk_compress_set_default_params(buf)
    off = _offsets()
    u8 = lambda k: buf.raw[off[k]]
    u32 = lambda k: int.from_bytes(buf.raw[off[k]:off[k] + 4], "little", signed=True)
    assert u8("numresolution") == 6 and u32("cblockw_init") == 64 and u32("cblockh_init") == 64
    assert u8("numgbits") == 2 and u32("roi_compno") == -1 and u32("subsampling_dx") == 1
    assert u32("prog_order") == 0 and u8("mct") == 0 and u32("repeats") == 1


_OFF = None


def _offsets():
    """grk_cparameters field offsets from the ABI header (compiled once)."""
    global _OFF
    if _OFF is None:
        import tempfile
        import pathlib
        with tempfile.TemporaryDirectory() as td:
            rows = _layout('#include "%s"' % ABI_H, {"grk_cparameters": _structs(ABI_H)["grk_cparameters"]},
                           pathlib.Path(td), "cp")
        _OFF = {r.split()[0].split(".")[-1]: int(r.split()[1]) for r in rows if "." in r.split(" ")[0]}
    return _OFF


def test_image_and_stream_objects_without_gpu():
    lib = _lib()
    lib.grk_image_new.restype = ctypes.c_void_p
    lib.grk_stream_create_mem_stream.restype = ctypes.c_void_p
    lib.grk_stream_get_write_mem_stream_length.restype = ctypes.c_size_t

    class Cmpt(ctypes.Structure):
        _fields_ = [(n, ctypes.c_uint32) for n in ("dx", "dy", "w", "stride", "h", "x0", "y0")] + \
                   [("prec", ctypes.c_uint8), ("sgnd", ctypes.c_bool)]
    parms = (Cmpt * 3)(*[Cmpt(1, 1, 17, 0, 9, 0, 0, 8, False) for _ in range(3)])
    img = lib.grk_image_new(3, parms, 2, True)
    assert img
    # grk_image: obj, x0, y0, x1, y1, numcomps ... comps (pointer at the end)
    raw = ctypes.string_at(img, 80)
    x1, y1 = int.from_bytes(raw[16:20], "little"), int.from_bytes(raw[20:24], "little")
    assert (x1, y1) == (17, 9)
    lib.grk_object_unref(ctypes.c_void_p(img))
    buf = ctypes.create_string_buffer(64)
    st = lib.grk_stream_create_mem_stream(buf, 64, False, False)
    assert st and lib.grk_stream_get_write_mem_stream_length(ctypes.c_void_p(st)) == 0
    lib.grk_object_unref(ctypes.c_void_p(st))
    # no separate plugin: "not handled" so callers take the regular path
    assert lib.grk_plugin_get_debug_state() == 0
    lib.grk_plugin_compress.restype = ctypes.c_int32
    assert lib.grk_plugin_compress(None, None) == -1
