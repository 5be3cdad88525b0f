"""Full-size BASELINE configs on the GPU vs reference Grok (tests/golden/full_size.json).

5/3 configs: the HIP encode of the seeded synthetic image must hash to the
exact SHA-256 of Grok 9.2.0's codestream, and decode back losslessly.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

FULL = json.load(open(os.path.join(GOLDEN, "full_size.json")))


def _img(cfg):
    from grok_amd.synth import synth_image
    img = synth_image(cfg["h"], cfg["w"], cfg["c"], cfg["bits"], cfg["seed"])
    assert hashlib.sha256(np.ascontiguousarray(img).tobytes()).hexdigest() == cfg["input_sha256"]
    return img.astype(np.int32)


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("name", ["C1", "C2", "C2p", "C4_4k", "C4_p1", "C4"])
def test_fullsize_lossless_bit_exact(eng, name):
    """C1/C2: Part 1 single tile; C4: 16384^2 16-bit HTJ2K, 1024^2 tiles, TLM + PLT
    (C4_4k / C4_p1: 4096^2 crops, HT and Part 1)."""
    import torch
    import grok_amd as G
    from conftest import parse_flags
    cfg = FULL[name]
    img = _img(cfg)
    kw = parse_flags(cfg["flags"])
    params = G.default_params(precincts=kw.get("precincts"), cblk_sty=kw.get("cblk_sty", 0), tiles=kw.get("tiles"),
                              tlm=kw.get("tlm", False), plt=kw.get("plt", False))
    x = torch.from_numpy(img).cuda()
    out = torch.empty(img.nbytes + (1 << 24), dtype=torch.uint8, device="cuda")
    n = eng.encode(x, cfg["bits"], params=params, out=out)
    assert n == cfg["bytes"]
    assert hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest() == cfg["sha256"]
    y = torch.empty_like(x)
    eng.decode(out, length=n, out=y)
    torch.cuda.synchronize()
    assert torch.equal(x, y)


@pytest.mark.parametrize("name", ["C3_l1", "C3_4k", "C3p"])
def test_fullsize_97_vs_grok(eng, name):
    """9/7 + ICT (+ PCRD layers): codestream SHA-256 equal to Grok's; our decode
    within the stated tolerance of Grok's decode PSNR."""
    import torch
    import grok_amd as G
    from conftest import parse_flags
    cfg = FULL[name]
    img = _img(cfg)
    kw = parse_flags(cfg["flags"])
    params = G.default_params(irreversible=True, precincts=kw.get("precincts"), layer_rate=kw.get("layer_rate"),
                              numlayers=len(kw.get("layer_rate") or [0]))
    x = torch.from_numpy(img).cuda()
    out = torch.empty(img.nbytes + (1 << 24), dtype=torch.uint8, device="cuda")
    n = eng.encode(x, cfg["bits"], params=params, out=out)
    cs = out[:n].cpu().numpy().tobytes()
    assert abs(n - cfg["bytes"]) <= 0.01 * cfg["bytes"]
    assert hashlib.sha256(cs).hexdigest() == cfg["sha256"]
    y = torch.empty_like(x)
    eng.decode(out, length=n, out=y)
    dec = y.cpu().numpy().astype(np.float64)
    mse = np.mean((dec - img) ** 2)
    psnr = 10 * np.log10(((1 << cfg["bits"]) - 1) ** 2 / mse)
    assert abs(psnr - cfg["grok_psnr_db"]) <= 0.1


def test_fullsize_c3_exact_config_vs_oracle(eng):
    """C3 exactly as BASELINE configures it (8192^2 RGB12, -I -r 40,20,10, single precinct):
    the reference is full_size.json C3: recorded from the oracle by make_oracle_fullsize.py
    and reproduced byte for byte by Grok 9.2.0's grk_compress in the round-3 review (Grok's
    decoder is broken on this stream, SURVEY R-BUG-3, so the decode is checked by PSNR)."""
    import torch
    import grok_amd as G
    cfg = FULL["C3"]
    img = _img(cfg)
    params = G.default_params(irreversible=True, layer_rate=[40.0, 20.0, 10.0])
    x = torch.from_numpy(img).cuda()
    out = torch.empty(img.nbytes + (1 << 24), dtype=torch.uint8, device="cuda")
    n = eng.encode(x, cfg["bits"], params=params, out=out)
    assert n == cfg["bytes"]
    assert hashlib.sha256(out[:n].cpu().numpy().tobytes()).hexdigest() == cfg["sha256"]
    y = torch.empty_like(x)
    eng.decode(out, length=n, out=y)
    dec = y.cpu().numpy().astype(np.float64)
    psnr = 10 * np.log10(4095.0 ** 2 / np.mean((dec - img) ** 2))
    assert psnr > 33.0   # the 3-layer stream decodes to ~33.4 dB (Grok's own decoder gives 17.9 dB here)
