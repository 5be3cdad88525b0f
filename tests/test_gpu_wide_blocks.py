"""Code-blocks with a side above 64 on the HIP path (128 x 32, 256 x 16, 512 x 8, 1024 x 4 and
their transposes; Part-1 and HTJ2K; encode and decode).

Grok accepts any 4 <= w, h <= 1024 with w * h <= 4096 (grk_compress.cpp:981-988) and sizes the
T1 state from the block (T1::alloc, T1.cpp:337-398).  Part-1 blocks of such streams run on the
lane-per-block coders of gk_t1ms.hip (state sized by the block), HT blocks on the wide-line
variants of k_ht_enc / k_ht_dec.  Bar: Grok's own codestreams (size and SHA-256, the round-5
review's known answers) byte for byte, seeded random shapes byte-equal to the oracle with
decodes, windows and rate control equal to the oracle's.
"""
import hashlib

import numpy as np
import pytest

import oracle as O
from conftest import parse_flags
from test_oracle_grok_sizes import IMAGES, KNOWN_WIDE

pytestmark = pytest.mark.gpu


def gk_params(kw):
    import grok_amd as G
    k = dict(kw)
    if "numres" in k:
        k["numresolution"] = k.pop("numres")
    if "layer_rate" in k:
        k["numlayers"] = len(k["layer_rate"])
    return G.default_params(**k)


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def images():
    from grok_amd.synth import synth_image
    return {k: (synth_image(*a).astype(np.int32), bits) for k, (a, bits) in IMAGES.items()}


@pytest.mark.parametrize("which,flags,grok_bytes,grok_sha", KNOWN_WIDE, ids=[k[1] for k in KNOWN_WIDE])
def test_wide_blocks_equal_grok(eng, images, which, flags, grok_bytes, grok_sha):
    import torch
    img, bits = images[which]
    kw = parse_flags(flags)
    cs = eng.encode(img, bits, params=gk_params(kw))
    assert len(cs) == grok_bytes
    assert hashlib.sha256(cs).hexdigest()[:16] == grok_sha
    want, _ = O.decode(cs)
    if "-r" not in flags:
        np.testing.assert_array_equal(want, img)
    np.testing.assert_array_equal(eng.decode(cs), want)
    dev = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    np.testing.assert_array_equal(eng.decode(dev, length=len(cs)), want)
    h, w = img.shape[1:]
    win = (w // 3 + 1, h // 4 + 3, w - 5, h - 7)
    np.testing.assert_array_equal(eng.decode_window(dev, win, length=len(cs)),
                                  O.decode(cs, partial=True)[0][:, win[1]:win[3], win[0]:win[2]])


SHAPES = [(128, 32), (256, 16), (512, 8), (1024, 4), (32, 128), (16, 256), (8, 512), (4, 1024), (128, 16), (256, 8)]


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    c = int(rng.choice([1, 3]))
    bits = int(rng.choice([8, 12, 16]))
    h, w = int(rng.integers(20, 400)), int(rng.integers(20, 600))
    from grok_amd.synth import synth_image
    img = synth_image(h, w, c, bits, 500 + seed).astype(np.int32)
    kw = {"numres": int(rng.integers(1, 7)), "cblk": SHAPES[seed % len(SHAPES)]}
    kind = seed % 5
    if kind == 1:
        kw["cblk_sty"] = 0x40                       # HTJ2K
    elif kind == 2:
        kw["cblk_sty"] = int(rng.choice([1, 2, 4, 8, 16, 32, 0x3f]))   # Part-1 mode switches
    if seed % 3 == 0:
        kw["tiles"] = (int(rng.integers(40, 300)), int(rng.integers(40, 300)))
    if seed % 4 == 1 and kind != 1:
        kw["layer_rate"] = [float(rng.choice([20, 40])), 5.0]
    if seed % 4 == 2:
        kw["irreversible"] = True
    if seed % 6 == 5:
        kw["precincts"] = [(256, 256), (128, 128)]
    return img, bits, kw


@pytest.mark.parametrize("seed", range(20))
def test_wide_blocks_random_vs_oracle(eng, seed):
    img, bits, kw = _case(seed)
    ref = O.encode(img, bits, **kw)
    cs = eng.encode(img, bits, params=gk_params(kw))
    assert cs == ref, ("codestream differs from oracle", kw, len(cs), len(ref))
    want, _ = O.decode(ref)
    np.testing.assert_array_equal(eng.decode(ref), want)
    if not kw.get("irreversible") and not kw.get("layer_rate"):
        np.testing.assert_array_equal(want, img)
    h, w = img.shape[1:]
    if h > 8 and w > 8:
        win = (w // 5, h // 3, w - w // 7, h - 2)
        np.testing.assert_array_equal(eng.decode_window(ref, win),
                                      O.decode(ref, partial=True)[0][:, win[1]:win[3], win[0]:win[2]])


def test_wide_blocks_refused_sizes(eng, images):
    # A.6.1: 4 <= side <= 1024 and w * h <= 4096 (xcb + ycb <= 12); Grok's CLI refuses the rest
    img, bits = images["A"]
    for cb in [(2048, 2), (128, 64), (2, 64)]:
        with pytest.raises(Exception):
            eng.encode(img, bits, params=gk_params({"cblk": cb}))
