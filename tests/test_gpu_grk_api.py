"""B1 drop-in on the GPU: a C program written against Grok's public API (tests/capi/
grk_api_roundtrip.c: the grk_compress / grk_decompress call sequence of src/bin) is
compiled against include/grk_abi.h, linked with libgrok_amd.so and run on every golden
fixture.  Its codestreams must equal Grok 9.2.0's byte for byte and its decodes must equal
Grok's decodes (source samples for lossless), through grk_image / grk_stream / grk_codec."""
import os
import subprocess

import numpy as np
import pytest

import grok_amd as G
import oracle as O
from conftest import FIXTURES, ROOT, fixture_ids

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tool(tmp_path_factory):
    d = tmp_path_factory.mktemp("capi")
    exe = str(d / "grk_api_roundtrip")
    subprocess.check_call(["gcc", "-std=c11", "-O1", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "capi", "grk_api_roundtrip.c"), "-o", exe,
                           "-L", os.path.dirname(G.LIB_PATH), "-lgrok_amd", "-Wl,-rpath," + os.path.dirname(G.LIB_PATH)])
    return exe, d


def _run(exe, *args):
    r = subprocess.run([exe] + [str(a) for a in args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    return r.stdout


def _enc(tool, img, bits, flags, name, extra=()):
    exe, d = tool
    raw = d / (name + ".raw")
    np.ascontiguousarray(img, dtype=np.int32).tofile(raw)
    c, h, w = img.shape
    out = d / (name + (".jp2" if "-jp2" in extra else ".j2k"))
    _run(exe, "enc", raw, w, h, c, bits, out, *flags.split(), *extra)
    return out.read_bytes(), out


def _dec(tool, path, shape, extra=()):
    exe, d = tool
    raw = d / (path.name + ".dec")
    info = _run(exe, "dec", path, raw, *extra)
    return np.fromfile(raw, np.int32).reshape(shape), info


@pytest.mark.parametrize("fx", FIXTURES, ids=fixture_ids(FIXTURES))
def test_grk_api_fixture_bit_exact(tool, fx):
    cs, path = _enc(tool, fx.img, fx.bits, fx.flags, fx.name)
    assert cs == fx.cs
    dec, info = _dec(tool, path, fx.img.shape)
    np.testing.assert_array_equal(dec, fx.grok_decoded if not fx.lossless else fx.img)
    assert "comps %d" % fx.img.shape[0] in info


@pytest.mark.parametrize("name", ["rgb8_tiles_xl", "mono16_ht_tiles", "rgb8_64"])
def test_grk_api_jp2_window_and_tiles(tool, name):
    fx = next(f for f in FIXTURES if f.name == name)
    cs, path = _enc(tool, fx.img, fx.bits, fx.flags, fx.name + "_jp2", extra=("-jp2",))
    assert cs == O.encode(fx.img, fx.bits, jp2=True, **fx.kw)          # JP2 boxes + Grok's codestream
    c, h, w = fx.img.shape
    x0, y0, x1, y1 = w // 5, h // 3, w - w // 7, h - 2
    dec, info = _dec(tool, path, (c, y1 - y0, x1 - x0), ("-d", "%d,%d,%d,%d" % (x0, y0, x1, y1)))
    np.testing.assert_array_equal(dec, fx.img[:, y0:y1, x0:x1])
    assert "image %d %d %d %d" % (x0, y0, x1, y1) in info
    if fx.tiled:
        tw, th = fx.kw["tiles"]
        t = 1
        tx0, ty0 = (t % ((w + tw - 1) // tw)) * tw, (t // ((w + tw - 1) // tw)) * th
        tdec, _ = _dec(tool, path, (c, min(th, h - ty0), min(tw, w - tx0)), ("-tile", t))
        np.testing.assert_array_equal(tdec, fx.img[:, ty0:ty0 + th, tx0:tx0 + tw])


@pytest.mark.parametrize("name", ["rgb8_tiles_xl", "mono16_ht_tiles", "rgb8_odd"])
def test_grk_api_compress_tile_raw_samples(tool, name):
    # grk_compress_tile with planar (prec + 7) / 8-byte tile buffers gives Grok's codestream
    fx = next(f for f in FIXTURES if f.name == name)
    cs, _ = _enc(tool, fx.img, fx.bits, fx.flags, fx.name + "_raw", extra=("-tiles",))
    assert cs == fx.cs
