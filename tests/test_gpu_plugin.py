"""B2 on the GPU: libgrokj2k_plugin.so driven through the plugin ABI by tests/capi/plugin_host.cpp,
which does what an unmodified Grok host does (loader, minpf registration, plugin_init; in the
compress callback it takes every code-block as compress_synch_with_plugin does,
plugin_bridge.cpp:146-270; in the decompress callback it plays grk_decompress's
decompress_callback, grk_decompress.cpp:996-1031).

Compress: the tree handed to the host must equal Grok's code-block state after T1 — per block
the geometry, bit-plane count, pass count, bytes, the pass rates the host derives and (rate
control) the distortion decreases — checked against the oracle (pinned to Grok's codestreams by
tests/test_oracle_golden.py), on every single-tile golden fixture.  Identical T1 state into
Grok's own T2 gives Grok's codestream.  Decompress: the image the plugin hands the host's
post-T1 stage equals Grok's decode (the source samples when lossless)."""
import os
import subprocess

import numpy as np
import pytest

import grok_amd as G
import oracle as O
from conftest import FIXTURES, ROOT, fixture_ids

pytestmark = pytest.mark.gpu
PLUGIN_DIR = os.path.dirname(G.LIB_PATH)
SINGLE = [f for f in FIXTURES if not f.tiled]


@pytest.fixture(scope="module")
def host(tmp_path_factory):
    d = tmp_path_factory.mktemp("plugin")
    exe = str(d / "plugin_host")
    subprocess.check_call(["g++", "-std=c++17", "-O1", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "capi", "plugin_host.cpp"), "-o", exe, "-ldl"])
    return exe, d


def _run(exe, *args):
    r = subprocess.run([exe, PLUGIN_DIR] + [str(a) for a in args], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, (r.returncode, r.stdout, r.stderr)
    return r.stdout


def write_pnm(path, img, bits):
    c, h, w = img.shape
    assert c in (1, 3)
    hdr = b"%s\n%d %d\n%d\n" % (b"P6" if c == 3 else b"P5", w, h, (1 << bits) - 1)
    px = np.ascontiguousarray(img.transpose(1, 2, 0))
    data = px.astype(">u2").tobytes() if bits > 8 else px.astype(np.uint8).tobytes()
    path.write_bytes(hdr + data)


def read_dump(path):
    b = path.read_bytes()
    out, i = [], 0
    while i < len(b):
        h = np.frombuffer(b, np.uint32, 15, i); i += 60
        n, ln = int(h[10]), int(h[11])
        rates = np.frombuffer(b, np.uint32, n, i); i += 4 * n
        dist = np.frombuffer(b, np.float64, n, i); i += 8 * n
        out.append((h.copy(), rates.copy(), dist.copy(), b[i:i + ln])); i += ln
    return out


@pytest.mark.parametrize("fx", SINGLE, ids=fixture_ids(SINGLE))
def test_plugin_encode_tree_matches_grok_t1(host, fx):
    exe, d = host
    pnm = d / (fx.name + (".ppm" if fx.img.shape[0] == 3 else ".pgm"))
    write_pnm(pnm, fx.img, fx.bits)
    dump = d / (fx.name + ".dump")
    out = _run(exe, "enc", pnm, dump, *fx.flags.split())
    assert "tree ok" in out
    got = read_dump(dump)
    blocks, data = O.encode_blocks(fx.img, fx.bits, **fx.kw)
    rates, dists = O.encode_block_passes(fx.img, fx.bits, **fx.kw)
    assert len(got) == len(blocks)
    q = 0
    for (h, r, dist, by), b in zip(got, blocks):
        want = [b.comp, b.res, b.band, b.prc, b.cblk, b.x0, b.y0, b.x1, b.y1, b.numbps, b.npasses, b.len]
        assert list(h[:12]) == want
        assert h[12] == (b.x1 - b.x0) * (b.y1 - b.y0)                       # numPix
        assert h[13] == (b.band + 1 if b.res else 0)                          # orientation
        assert by == data[b.data_off:b.data_off + b.len].tobytes()
        np.testing.assert_array_equal(r, rates[q:q + b.npasses])              # host-derived pass rates
        # rate control: cumulative distortion decrease in f64; the GPU sum may differ from the
        # oracle's in the last place (the PCRD result does not: the fixture codestreams are
        # byte-identical to Grok's, tests/test_gpu_parity.py)
        np.testing.assert_allclose(dist, dists[q:q + b.npasses], rtol=1e-13, atol=0)
        q += b.npasses


@pytest.mark.parametrize("fx", FIXTURES, ids=fixture_ids(FIXTURES))
def test_plugin_decompress(host, fx):
    exe, d = host
    cs = d / (fx.name + ".j2k")
    cs.write_bytes(fx.cs)
    raw = d / (fx.name + ".raw")
    out = _run(exe, "dec", cs, raw)
    assert "stages header post(plugin image) clean" in out
    dec = np.fromfile(raw, np.int32).reshape(fx.img.shape)
    np.testing.assert_array_equal(dec, fx.img if fx.lossless else fx.grok_decoded)


def test_plugin_decompress_window(host):
    fx = next(f for f in FIXTURES if f.name == "rgb8_odd")
    exe, d = host
    cs = d / "win.j2k"
    cs.write_bytes(fx.cs)
    raw = d / "win.raw"
    out = _run(exe, "dec", cs, raw, "-d", "17,9,200,120")
    assert "image 17 9 200 120 comps 3" in out
    dec = np.fromfile(raw, np.int32).reshape(3, 111, 183)
    np.testing.assert_array_equal(dec, fx.img[:, 9:120, 17:200])


def test_plugin_refuses_tiles(host):
    # the plugin tile is one tile: a multi-tile request is "not handled" (-1), so Grok keeps its CPU path
    fx = next(f for f in FIXTURES if f.name == "rgb8_tiles")
    exe, d = host
    pnm = d / "tiles.ppm"
    write_pnm(pnm, fx.img, fx.bits)
    r = subprocess.run([exe, PLUGIN_DIR, "enc", pnm, d / "tiles.dump", "-t", "128,128"], capture_output=True,
                       text=True, timeout=120)
    assert "plugin_encode rc -1 blocks 0" in r.stdout, (r.stdout, r.stderr)
