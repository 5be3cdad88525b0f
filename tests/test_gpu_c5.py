"""C5 at full size (BASELINE configs[4]): a 32768x32768 RGB8 tiled .jp2 (1024x1024 tiles,
TLM + PLT; grk_compress -t 1024,1024 -X -L, .jp2 output), random-window decode.

The file is built on the GPU tile row by tile row from planar u8 slabs
(grok_amd.bigimage) and must hash to full_size.json "C5": first recorded from the oracle,
then reproduced byte for byte by Grok 9.2.0's own grk_compress in the round-3 review.  The four SURVEY windows are decoded from the device-resident
file (TLM finds the tiles, PLT the packets; code-blocks out of the window's reach are
skipped) and must equal the source samples exactly (lossless)."""
import hashlib
import json
import os

import numpy as np
import pytest
import torch

import grok_amd as G
from grok_amd import bigimage
from conftest import GOLDEN

pytestmark = pytest.mark.gpu

REF = json.load(open(os.path.join(GOLDEN, "full_size.json"))).get("C5")
OUT = os.path.join(os.path.dirname(GOLDEN), "..", "gpurun_out")


def _progress(done, total):
    os.makedirs(OUT, exist_ok=True)
    with open(os.path.join(OUT, "c5_progress.log"), "a") as f:
        f.write("C5 rows %d / %d\n" % (done, total))


@pytest.fixture(scope="module")
def c5():
    if REF is None:
        pytest.skip("no C5 reference in full_size.json")
    eng = G.Engine(0)
    p = G.default_params(tiles=(1024, 1024), tlm=True, plt=True, jp2=True)
    crops = {k: tuple(v["rect"]) for k, v in REF["windows"].items()}
    it = bigimage.slabs(REF["h"], REF["w"], REF["c"], REF["bits"], REF["seed"], 1024, threads=16)
    f, n, src = bigimage.encode_tiled(eng, (REF["c"], REF["h"], REF["w"]), REF["bits"], p, it, torch.device("cuda", 0),
                                      crops=crops, progress=_progress)
    yield eng, f, n, src
    eng.close()


@pytest.mark.timeout(900)
def test_c5_file_matches_oracle(c5):
    eng, f, n, src = c5
    assert n == REF["bytes"]
    assert hashlib.sha256(f.cpu().numpy().tobytes()).hexdigest() == REF["sha256"]


@pytest.mark.timeout(900)
@pytest.mark.parametrize("name", ["w1k_origin", "w4k_unaligned", "w_edge", "w16k"])
def test_c5_window_decode_exact(c5, name):
    eng, f, n, src = c5
    x0, y0, x1, y1 = REF["windows"][name]["rect"]
    assert hashlib.sha256(src[name].tobytes()).hexdigest() == REF["windows"][name]["source_sha256"]
    y = torch.empty((3, y1 - y0, x1 - x0), dtype=torch.uint8, device="cuda")
    eng.decode_window(f, (x0, y0, x1, y1), length=n, out=y)
    np.testing.assert_array_equal(y.cpu().numpy(), src[name])


@pytest.mark.timeout(900)
def test_c5_window_from_host_file(c5):
    # host bytes without the device: SOT walk over the 1024 tile parts
    eng, f, n, src = c5
    host = f[:n].cpu().numpy().tobytes()
    x0, y0, x1, y1 = REF["windows"]["w_edge"]["rect"]
    np.testing.assert_array_equal(eng.decode_window(host, (x0, y0, x1, y1), sample_bytes=1), src["w_edge"])
