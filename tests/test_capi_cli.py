"""B1 with the unchanged src/bin call sequences, on a host without a GPU.

tests/capi/grk_api_roundtrip.c makes the exact grk_* call sequences of Grok's own tools:
grk_compress (pluginMain grk_compress.cpp:2171-2213, compress() :2055-2156), grk_decompress
(pluginMain grk_decompress.cpp:897-921, preProcess :1041-1295 with its unconditional
grk_decompress_set_window at :1259) and grk_dump (grk_dump.cpp:342-504).  Here, without a GPU,
every sequence must get through the API to the engine call and stop there with the engine's
refusal ("no HIP device"), never at an API error; grk_dump needs no engine and must complete.
The same harness runs end to end on the GPU in tests/test_gpu_grk_api.py.
"""
import os
import subprocess

import numpy as np
import pytest

import grok_amd as G
from conftest import FIXTURES, ROOT

REFUSAL = "no HIP device"


@pytest.fixture(scope="module")
def tool(tmp_path_factory):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: tests/test_gpu_grk_api.py runs these sequences end to end")
    G.load_library()
    d = tmp_path_factory.mktemp("capi_cli")
    exe = str(d / "grk_api_roundtrip")
    subprocess.check_call(["gcc", "-std=c11", "-O1", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "capi", "grk_api_roundtrip.c"), "-o", exe,
                           "-L", os.path.dirname(G.LIB_PATH), "-lgrok_amd",
                           "-Wl,-rpath," + os.path.dirname(G.LIB_PATH)])
    return exe, d


def _run(exe, *args):
    return subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True, timeout=60)


def _fx(name):
    return next(f for f in FIXTURES if f.name == name)


def _stream(tool, name, ext=".j2k"):
    exe, d = tool
    p = d / (name + ext)
    p.write_bytes(_fx(name).cs)
    return p


def test_dump_completes_without_gpu(tool):
    exe, _ = tool
    fx = _fx("rgb8_tiles_xl")
    r = _run(exe, "dump", _stream(tool, fx.name))
    assert r.returncode == 0, r.stderr
    c, h, w = fx.img.shape
    assert "x1=%d, y1=%d" % (w, h) in r.stdout and "numcomps=%d" % c in r.stdout
    assert "tdx=128, tdy=128" in r.stdout and "numresolutions=6" in r.stdout


@pytest.mark.parametrize("extra", [(), ("-d", "0,0,0,0"), ("-mapped",), ("-l", "1")])
def test_decompress_full_image_reaches_engine(tool, extra):
    # no -d: the CLI still calls set_window(0,0,0,0), which means the whole image
    # (CodeStreamDecompress.cpp:309-316)
    exe, d = tool
    r = _run(exe, "dec", _stream(tool, "rgb8_tiles_xl"), d / "o.raw", *extra)
    assert r.returncode == 9, (r.returncode, r.stdout, r.stderr)    # grk_decompress, not set_window (8)
    assert REFUSAL in r.stderr and "header cblk 64x64" in r.stdout


def test_decompress_window_clamps_right_bottom(tool):
    # right / bottom past the image: warning and clamp (CodeStreamDecompress.cpp:355-388)
    exe, d = tool
    r = _run(exe, "dec", _stream(tool, "rgb8_tiles_xl"), d / "o.raw", "-d", "10,20,5000,6000")
    assert r.returncode == 9, (r.returncode, r.stderr)
    assert "Right position of the decompress window (5000)" in r.stderr
    assert "Bottom position of the decompress window (6000)" in r.stderr
    assert REFUSAL in r.stderr


def test_decompress_window_left_top_outside_is_error(tool):
    # left / top past the image: error (CodeStreamDecompress.cpp:325-350)
    exe, d = tool
    fx = _fx("rgb8_tiles_xl")
    c, h, w = fx.img.shape
    r = _run(exe, "dec", _stream(tool, fx.name), d / "o.raw", "-d", "%d,0,%d,10" % (w + 1, w + 50))
    assert r.returncode == 8 and "Left position" in r.stderr
    r = _run(exe, "dec", _stream(tool, fx.name), d / "o.raw", "-d", "0,%d,10,%d" % (h + 1, h + 50))
    assert r.returncode == 8 and "Top position" in r.stderr


def test_decompress_tile_reaches_engine(tool):
    exe, d = tool
    r = _run(exe, "dec", _stream(tool, "rgb8_tiles_xl"), d / "o.raw", "-tile", "1")
    assert r.returncode == 7 and REFUSAL in r.stderr, (r.returncode, r.stderr)
    r = _run(exe, "dec", _stream(tool, "rgb8_tiles_xl"), d / "o.raw", "-tile", "99")
    assert r.returncode == 7 and "greater than maximum tile index" in r.stderr


@pytest.mark.parametrize("name,extra", [("rgb8_tiles_xl", ()), ("rgb12_97_r", ()), ("mono16_ht_tiles", ()),
                                        ("rgb8_64", ("-jp2",)), ("rgb8_64", ("-file",)),
                                        ("rgb8_tiles", ("-tiles",))])
def test_compress_reaches_engine(tool, name, extra):
    exe, d = tool
    fx = _fx(name)
    raw = d / (name + ".raw")
    np.ascontiguousarray(fx.img, dtype=np.int32).tofile(raw)
    c, h, w = fx.img.shape
    r = _run(exe, "enc", raw, w, h, c, fx.bits, d / (name + ".out"), *fx.flags.split(), *extra)
    assert r.returncode == 5, (r.returncode, r.stdout, r.stderr)    # the compress call, after init/start (4)
    assert REFUSAL in r.stderr
