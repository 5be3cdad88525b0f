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


def test_grk_api_cli_window_semantics(tool):
    # grk_decompress.cpp:1259 calls set_window with the -d values or zeros: (0,0,0,0) is the
    # whole image; right / bottom edges past the image clamp with a warning
    # (CodeStreamDecompress.cpp:309-316, :355-388); the composited image pointer taken after
    # the header read is the one decoded into
    fx = next(f for f in FIXTURES if f.name == "rgb8_tiles_xl")
    cs, path = _enc(tool, fx.img, fx.bits, fx.flags, fx.name + "_cli")
    c, h, w = fx.img.shape
    dec, _ = _dec(tool, path, fx.img.shape, ("-d", "0,0,0,0"))
    np.testing.assert_array_equal(dec, fx.img)
    x0, y0 = 17, 33
    dec, info = _dec(tool, path, (c, h - y0, w - x0), ("-d", "%d,%d,%d,%d" % (x0, y0, w + 100, h + 7)))
    np.testing.assert_array_equal(dec, fx.img[:, y0:, x0:])
    assert "image %d %d %d %d" % (x0, y0, w, h) in info
    # a tile decode crops the composited image to the tile, intersected with the window
    tw, th = fx.kw["tiles"]
    dec, info = _dec(tool, path, (c, th - 5, tw - 9), ("-tile", 0, "-d", "9,5,%d,%d" % (w, h)))
    np.testing.assert_array_equal(dec, fx.img[:, 5:th, 9:tw])


@pytest.mark.parametrize("name,red,layers", [("rgb8_64", 2, 0), ("rgb12_97_r", 1, 2), ("rgb8_tiles_xl", 1, 0)])
def test_grk_api_cli_reduce_and_layers(tool, name, red, layers):
    # -r / -l through grk_dparameters (cp_reduce, cp_layer), with the CLI's set_window(0,0,0,0)
    fx = next(f for f in FIXTURES if f.name == name)
    exe, d = tool
    p = d / (name + "_rl.j2k")
    p.write_bytes(fx.cs)
    c, h, w = fx.img.shape
    shape = (c, (h + (1 << red) - 1) >> red, (w + (1 << red) - 1) >> red)
    dec, _ = _dec(tool, p, shape, ("-r", red, "-l", layers))
    O.set_decode_reduce(red)
    O.set_decode_layers(layers)
    try:
        want, _ = O.decode(fx.cs)
    finally:
        O.set_decode_reduce(0)
        O.set_decode_layers(0)
    np.testing.assert_array_equal(dec, want)


@pytest.mark.parametrize("name,red", [("rgb8_tiles_xl", 1), ("rgb12_97_r", 2)])
def test_grk_api_cli_reduce_window(tool, name, red):
    # -r with -d: the window's canvas rectangle on the reduced canvas (ceil(x / 2^r) per edge,
    # CodeStreamDecompress.cpp:471-481), decoded under the partial-tile rule a window selects
    fx = next(f for f in FIXTURES if f.name == name)
    exe, d = tool
    p = d / (name + "_rw.j2k")
    p.write_bytes(fx.cs)
    c, h, w = fx.img.shape
    x0, y0, x1, y1 = 17, 33, w - 5, h - 3
    cd = lambda v: -(-v >> red)
    dec, info = _dec(tool, p, (c, cd(y1) - cd(y0), cd(x1) - cd(x0)), ("-r", red, "-d", "%d,%d,%d,%d" % (x0, y0, x1, y1)))
    O.set_decode_reduce(red)
    try:
        want, _ = O.decode(fx.cs, partial=True)
    finally:
        O.set_decode_reduce(0)
    np.testing.assert_array_equal(dec, want[:, cd(y0):cd(y1), cd(x0):cd(x1)])
    assert "image %d %d %d %d" % (x0, y0, x1, y1) in info   # (the image keeps its full-resolution bounds)
    if fx.tiled:   # -r with -tile: the tile's rectangle reduced the same way
        tw, th = fx.kw["tiles"]
        tx0, ty0, tx1, ty1 = tw, 0, min(2 * tw, w), min(th, h)
        dec, _ = _dec(tool, p, (c, cd(ty1) - cd(ty0), cd(tx1) - cd(tx0)), ("-r", red, "-tile", 1))
        np.testing.assert_array_equal(dec, want[:, cd(ty0):cd(ty1), cd(tx0):cd(tx1)])


@pytest.mark.parametrize("flags", ["-S -E", "-S -r 20,5", "-q 30,40", "-E -q 28,36,0 -t 128,128 -X"])
def test_grk_api_sop_eph_quality(tool, flags):
    # grk_compress -S / -E / -q through grk_cparameters (csty, allocationByQuality, layer_distortion)
    from grok_amd.synth import synth_image
    img = synth_image(200, 300, 3, 8, 77).astype(np.int32)
    cs, path = _enc(tool, img, 8, flags, "sq_" + flags.replace(" ", "_").replace(",", "_"))
    from conftest import parse_flags
    assert cs == O.encode(img, 8, **parse_flags(flags))
    dec, _ = _dec(tool, path, img.shape)
    want, _ = O.decode(cs)
    np.testing.assert_array_equal(dec, want)


@pytest.mark.parametrize("flags", ["-r 20,10,5 -P T0=0,0,1,3,3,RLCP/T0=3,0,3,6,3,LRCP/T0=0,0,3,6,3,RPCL",
                                   "-p CPRL -c [64,64],[32,32]", "-n 4 -P T0=0,0,1,4,3,PCRL/T0=0,0,1,5,3,LRCP"])
def test_grk_api_progression_changes(tool, flags):
    # grk_cparameters::progression / numpocs (grk_compress -P) and prog_order (-p)
    from grok_amd.synth import synth_image
    img = synth_image(160, 224, 3, 8, 78).astype(np.int32)
    cs, path = _enc(tool, img, 8, flags, "poc_%d" % (abs(hash(flags)) % 10000))
    from conftest import parse_flags
    assert cs == O.encode(img, 8, **parse_flags(flags))
    dec, _ = _dec(tool, path, img.shape)
    want, _ = O.decode(cs)
    np.testing.assert_array_equal(dec, want)


@pytest.mark.parametrize("flags", ["-d 17,9 -T 5,2 -t 32,48", "-T 7,3 -t 40,40", "-d 3,5", "-d 65,33 -T 64,32 -t 32,32 -X -L"])
def test_grk_api_offsets(tool, flags):
    # grk_compress -d (image offset: grk_image::x0 / y0) and -T (grk_cparameters::tx0 / ty0)
    from grok_amd.synth import synth_image
    img = synth_image(90, 110, 3, 8, 79).astype(np.int32)
    cs, path = _enc(tool, img, 8, flags, "off_%d" % (abs(hash(flags)) % 10000))
    from conftest import parse_flags
    assert cs == O.encode(img, 8, **parse_flags(flags))
    dec, _ = _dec(tool, path, img.shape)
    np.testing.assert_array_equal(dec, img)


def test_grk_api_tile_rule_without_window(tool):
    # grk_decompress -tile t with no -d decodes the tile with Grok's whole-tile
    # inverse (decompressTile keeps wholeTileDecompress), a -d window with the partial-tile one;
    # the fixture makes the two rules differ inside tile 3 (tests/window_rule_case.py)
    from window_rule_case import LAYERS, TILE, case
    img, kw = case()
    cs = O.encode(img, 8, **kw)
    exe, d = tool
    p = d / "tile_rule.j2k"
    p.write_bytes(cs)
    O.set_decode_layers(LAYERS)
    try:
        whole, _ = O.decode(cs)
        part, _ = O.decode(cs, partial=True)
    finally:
        O.set_decode_layers(0)
    tw, h = kw["tiles"]
    x0, x1 = TILE * tw, min((TILE + 1) * tw, img.shape[2])
    assert (whole[:, :, x0:x1] != part[:, :, x0:x1]).any()
    dec, _ = _dec(tool, p, (1, h, x1 - x0), ("-tile", TILE, "-l", LAYERS))
    np.testing.assert_array_equal(dec, whole[:, :, x0:x1])
    dec, _ = _dec(tool, p, (1, h, x1 - x0), ("-d", "%d,0,%d,%d" % (x0, x1, h), "-l", LAYERS))
    np.testing.assert_array_equal(dec, part[:, :, x0:x1])
    dec, _ = _dec(tool, p, (1, h, x1 - x0), ("-tile", TILE, "-d", "%d,0,%d,%d" % (x0, x1, h), "-l", LAYERS))
    np.testing.assert_array_equal(dec, part[:, :, x0:x1])
    dec, _ = _dec(tool, p, img.shape, ("-l", LAYERS))
    np.testing.assert_array_equal(dec, whole)


@pytest.mark.parametrize("flags,grok_bytes,grok_sha", [("-b 128,32", 410963, "69f2f8af6486a243"),
                                                       ("-b 1024,4 -r 20,5", 119723, "e7f7599fcd9dc5ef")])
def test_grk_api_wide_code_blocks(tool, flags, grok_bytes, grok_sha):
    # grk_compress -b W,H with a side above 64 (grk_compress.cpp:981-988) through the drop-in
    import hashlib
    from grok_amd.synth import synth_image
    img = synth_image(384, 520, 3, 8, 7).astype(np.int32)
    cs, path = _enc(tool, img, 8, flags, "wide_" + flags.split()[1].replace(",", "x"))
    assert len(cs) == grok_bytes and hashlib.sha256(cs).hexdigest()[:16] == grok_sha
    dec, _ = _dec(tool, path, img.shape)
    want, _ = O.decode(cs)
    np.testing.assert_array_equal(dec, want)


@pytest.mark.parametrize("name, flags", [("420_53", "-n 3"), ("tiled_pcrl", "-n 3 -t 64,32 -p PCRL -c [16,16]"),
                                         ("422_97", "-n 4 -I")])
def test_grk_api_subsampled_components(tool, name, flags):
    # an API user's grk_image with subsampled components (grk_image_comp dx / dy): the shim codes
    # the oracle's bytes and decodes each component at its own size (the CLI's raw reader itself
    # refuses subsampling, RAWFormat.cpp:293-298, so this is the library-level call sequence)
    from subsampling_cases import CASES, planes, oracle_kw
    W, H, sub, prec, kw = CASES[name]
    exe, d = tool
    src = planes(name)
    raw = d / (name + "_sub.raw")
    np.concatenate([p.ravel() for p in src]).astype(np.int32).tofile(raw)
    out = d / (name + "_sub.j2k")
    subarg = ":".join("%dx%d" % s for s in sub)
    _run(exe, "enc", raw, W, H, len(sub), prec, out, *flags.split(), "-sub", subarg)
    ref = O.encode(src, prec, size=(W, H), **oracle_kw(name))
    assert out.read_bytes() == ref
    dec = d / (name + "_sub.dec")
    _run(exe, "dec", out, dec)
    flat = np.fromfile(dec, np.int32)
    want, _ = O.decode(ref)
    np.testing.assert_array_equal(flat, np.concatenate([w.ravel() for w in want]))


def test_grk_api_subsampled_window(tool):
    # grk_decompress -d on a 4:2:0 stream: each component of the composite takes the window's
    # rectangle on its grid (GrkImage::subsampleAndReduce), decoded with the partial-tile rule
    from subsampling_cases import CASES, planes, oracle_kw
    name = "tiled_pcrl"
    W, H, sub, prec, kw = CASES[name]
    exe, d = tool
    ref = O.encode(planes(name), prec, size=(W, H), **oracle_kw(name))
    path = d / "sub_win.j2k"
    path.write_bytes(ref)
    x0, y0, x1, y1 = 9, 5, 101, 63
    dec = d / "sub_win.dec"
    _run(exe, "dec", path, dec, "-d", "%d,%d,%d,%d" % (x0, y0, x1, y1))
    full, _ = O.decode(ref, partial=True)
    want = []
    for f, (dx, dy) in zip(full, sub):
        cd = lambda a, b: -(-a // b)
        want.append(f[cd(y0, dy):cd(y1, dy), cd(x0, dx):cd(x1, dx)].ravel())
    np.testing.assert_array_equal(np.fromfile(dec, np.int32), np.concatenate(want))


@pytest.mark.parametrize("flags", ["-n 4", "-n 5 -r 40,10"])
def test_grk_api_comments(tool, flags):
    # grk_compress -C "a|b": COM markers instead of Grok's default one; with rate control the
    # header's extra bytes move the layer budgets (updateRates' header size), as in Grok
    from grok_amd.synth import synth_image
    from conftest import parse_flags
    img = synth_image(96, 120, 3, 8, 31).astype(np.int32)
    cs, _ = _enc(tool, img, 8, flags, "com_%d" % len(flags), extra=("-C", "first|second comment"))
    ref = O.encode(img, 8, comments=["first", "second comment"], **parse_flags(flags))
    assert cs == ref
    assert cs.count(b"\xff\x64") == 2 and b"Created by Grok" not in cs


@pytest.mark.parametrize("kind", ["tile_coding", "coc", "ppm"])
def test_grk_api_third_party_streams(tool, kind):
    # grk_decompress's call sequence on streams Grok's encoder never writes but its decoder reads:
    # tiles with their own coding (tile-part COD / QCD), per-component COC / QCC, PPM packed
    # headers; the shim returns the oracle's samples, also through -tile (Grok's whole-tile rule)
    exe, d = tool
    if kind == "tile_coding":
        import tile_coding
        cs = tile_coding.stream("levels_cblk")
    elif kind == "coc":
        import test_coc
        cs = test_coc.stream("levels_cblk_97_prc")
    else:
        import test_ppx
        cs = test_ppx.stream("tiles_sop_eph", "ppm")
    path = d / ("third_%s.j2k" % kind)
    path.write_bytes(cs)
    dec = d / ("third_%s.dec" % kind)
    _run(exe, "dec", path, dec)
    want, _ = O.decode(cs)
    want = want if isinstance(want, list) else list(want)
    np.testing.assert_array_equal(np.fromfile(dec, np.int32), np.concatenate([w.ravel() for w in want]))
    if kind == "tile_coding":   # tile 1 (B-coded) alone
        import tile_coding
        x0, y0, x1, y1 = tile_coding.tile_rects("levels_cblk")[1]
        _run(exe, "dec", path, dec, "-tile", "1")
        full = tile_coding.expected("levels_cblk")
        np.testing.assert_array_equal(np.fromfile(dec, np.int32), full[:, y0:y1, x0:x1].ravel())
