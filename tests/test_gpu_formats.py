"""GPU parity for the data formats either side of the hot path: the JP2 file format
(FileFormatCompress / FileFormatDecompress), planar 8/16-bit sample ingest and egress
(TileProcessor::ingestUncompressedData), and window decode with code-block / packet
skipping (T2Decompress.cpp:55-116).  The oracle (CPU restatement, Grok-pinned) is the
checker; windows of lossless streams must equal the source crop."""
import numpy as np
import pytest
import torch

import grok_amd as G
import oracle as O
from grok_amd.synth import synth_image

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    e = G.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("kw", [dict(), dict(tiles=(64, 64), tlm=True, plt=True), dict(irreversible=True),
                                dict(cblk_sty=0x40, tiles=(128, 64), tlm=True, plt=True)])
def test_jp2_encode_matches_oracle(eng, kw):
    img = synth_image(150, 230, 3, 8, 31).astype(np.int32)
    ref = O.encode(img, 8, jp2=True, **kw)
    cs = eng.encode(img, 8, params=G.default_params(jp2=True, **kw))
    assert cs == ref
    dec = eng.decode(cs)
    if not kw.get("irreversible"):
        np.testing.assert_array_equal(dec, img)
    d = torch.from_numpy(np.frombuffer(cs, np.uint8).copy()).cuda()
    y = torch.empty(img.shape, dtype=torch.int32, device="cuda")
    eng.decode(d, length=len(cs), out=y)
    np.testing.assert_array_equal(y.cpu().numpy(), dec)


def test_jp2_xl_box_for_large_raw_images(eng):
    # raw image > 2^30 bytes: jp2c header carries the 8-byte XLBox (FileFormatCompress.cpp:678-686)
    hdr = eng.jp2_header((3, 32768, 32768), 8, 1000)
    assert hdr == O.jp2_header(32768, 32768, 3, 8, 1000)


@pytest.mark.parametrize("bits,comps,signed", [(8, 3, False), (8, 1, True), (12, 3, False), (16, 1, False),
                                               (16, 1, True)])
def test_sample_ingest_egress(eng, bits, comps, signed):
    # planar (prec + 7) / 8-byte samples in, same out: identical codestream to int32 planes
    h, w = 97, 130
    img = synth_image(h, w, comps, bits, 32).astype(np.int64)
    if signed:
        img -= 1 << (bits - 1)
    dt = {(8, False): np.uint8, (8, True): np.int8, (16, False): np.uint16, (16, True): np.int16}[
        ((bits + 7) // 8 * 8, signed)]
    small = img.astype(dt)
    kw = dict(tiles=(64, 64)) if comps == 1 else dict()
    p = G.default_params(**kw)
    ref = eng.encode(img.astype(np.int32), bits, signed=signed, params=p)
    assert eng.encode(small, bits, signed=signed, params=p) == ref                     # host 8/16-bit planes
    tdt = {np.uint8: torch.uint8, np.int8: torch.int8, np.uint16: torch.int16, np.int16: torch.int16}[dt]
    x = torch.from_numpy(small.view(np.int16) if dt == np.uint16 else small).cuda()
    out = torch.empty(small.nbytes * 2 + 4096, dtype=torch.uint8, device="cuda")
    n = eng.encode(x, bits, signed=signed, params=p, out=out)                         # device 8/16-bit planes
    assert out[:n].cpu().numpy().tobytes() == ref
    dec = eng.decode(ref, sample_bytes=small.itemsize)
    assert dec.dtype == dt
    np.testing.assert_array_equal(dec, small)
    y = torch.empty(x.shape, dtype=tdt, device="cuda")
    eng.decode(out, length=n, out=y)
    np.testing.assert_array_equal(y.cpu().numpy().view(dt), small)


WINDOWS = [(0, 0, 64, 64), (1, 1, 2, 2), (37, 81, 38, 300), (63, 63, 65, 65), (100, 17, 261, 190), (250, 0, 263, 201)]


@pytest.mark.parametrize("kw", [dict(tiles=(64, 64), tlm=True, plt=True),
                                dict(tiles=(128, 128), tlm=True, plt=True, precincts=[(32, 32)], cblk=(16, 16)),
                                dict(tiles=(128, 64), plt=True, irreversible=True),
                                dict(tiles=(64, 128), tlm=True, plt=True, cblk_sty=0x40),
                                dict(precincts=[(64, 64), (32, 32)], cblk=(32, 32), plt=True),
                                dict(irreversible=True, precincts=[(64, 64)], plt=True)])
def test_window_decode_skips_blocks_exactly(eng, kw):
    # windows smaller than a tile: code-blocks (and, with PLT and precincts, whole packets)
    # outside the window's reach are skipped; the window equals the crop of the full decode
    img = synth_image(201, 263, 3, 8, 33).astype(np.int32)
    cs = O.encode(img, 8, jp2=True, **kw)
    full = eng.decode(cs)
    if not kw.get("irreversible"):
        np.testing.assert_array_equal(full, img)
    d = torch.from_numpy(np.frombuffer(cs, np.uint8).copy()).cuda()
    for (x0, y0, x1, y1) in WINDOWS:
        x1, y1 = min(x1, 263), min(y1, 201)
        np.testing.assert_array_equal(eng.decode_window(cs, (x0, y0, x1, y1)), full[:, y0:y1, x0:x1])
        y = torch.empty((3, y1 - y0, x1 - x0), dtype=torch.uint8, device="cuda")
        eng.decode_window(d, (x0, y0, x1, y1), length=len(cs), out=y)
        np.testing.assert_array_equal(y.cpu().numpy(), full[:, y0:y1, x0:x1].astype(np.uint8))
    eng.decode(cs)   # a full decode after windows still works (per-call regions)
