"""The C-ABI boundary (include/grok_amd.h) without a GPU.

Checks that the in-tree HIP extension loads, exports every entry point the
header declares, that the ctypes mirror of the structs matches the C layout,
and that the product fails loudly (no CPU fallback) when no GPU is present.
"""
import ctypes
import os
import re
import subprocess
import tempfile

import pytest

from conftest import ROOT
import grok_amd as G

HEADERS = [os.path.join(ROOT, "include", f) for f in os.listdir(os.path.join(ROOT, "include")) if f.endswith(".h")]


def declared_symbols():
    syms = set()
    for h in HEADERS:
        txt = open(h).read()
        txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w\s\*]*?\b((?:gk|grk)_\w+)\s*\(", txt, flags=re.M):
            syms.add(m.group(1))
    return syms


def test_library_builds_and_loads():
    lib = G.load_library()
    assert lib.gk_version().decode().startswith("grok_amd")


def test_every_declared_symbol_is_exported():
    syms = declared_symbols()
    assert "gk_encode" in syms and "gk_decode" in syms
    out = subprocess.run(["nm", "-D", "--defined-only", G.LIB_PATH], capture_output=True, text=True, check=True).stdout
    exported = {l.split()[-1] for l in out.splitlines() if l.strip()}
    missing = sorted(s for s in syms if s not in exported)
    assert not missing, missing
    assert set(G.EXPORTS) <= exported


def test_struct_layout_matches_header(tmp_path):
    src = tmp_path / "layout.c"
    src.write_text('#include "grok_amd.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                   'int main(void){printf("%zu %zu %zu %zu %zu %zu %zu\\n", sizeof(gk_cparameters), sizeof(gk_image_info),'
                   ' sizeof(gk_timings), offsetof(gk_cparameters, write_comment), offsetof(gk_timings, dwt_bytes),'
                   ' offsetof(gk_cparameters, cod_format), offsetof(gk_image_info, sample_bytes));'
                   'return 0;}\n')
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)])
    got = [int(v) for v in subprocess.check_output([str(exe)]).split()]
    want = [ctypes.sizeof(G.CParameters), ctypes.sizeof(G.ImageInfo), ctypes.sizeof(G.Timings),
            G.CParameters.write_comment.offset, G.Timings.dwt_bytes.offset, G.CParameters.cod_format.offset,
            G.ImageInfo.sample_bytes.offset]
    assert got == want


def test_no_cpu_fallback_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(RuntimeError, match="no HIP device"):
        G.Engine(0)


def test_default_params_mirror_grok_defaults():
    # grk_compress_set_default_params (grok.cpp:405-435): 6 resolutions, 64x64 blocks, 1 layer, 2 guard bits
    p = G.default_params()
    assert p.numresolution == 6 and p.cblockw_init == 64 and p.cblockh_init == 64
    assert p.numlayers == 1 and p.numgbits == 2 and p.irreversible == 0
    # the C API default leaves the MCT off (memset, grok.cpp:409); the CLI switches it on for RGB
    raw = G.CParameters()
    G.load_library().gk_set_default_params(ctypes.byref(raw))
    assert raw.mct == 0 and raw.cod_format == 0 and raw.numresolution == 6
