"""The HIP engine on Grok 9.2.0's known answers (tests/test_oracle_grok_sizes.py: size and
SHA-256 of Grok's own grk_compress output, recorded by the reviews): tiled rate control, mode
switches and precincts with tiles, tile-part generation with rates, odd-parity tiles, POC.

Encode: byte-equal to the oracle and to Grok's hash.  Decode: the streams with Grok's
simulation-counted Psot / TLM / PLT decode like the oracle's decode, from
host and from device memory (the TLM path), whole and through a window (PLT path).
"""
import hashlib

import numpy as np
import pytest

import oracle as O
from conftest import parse_flags
from test_oracle_grok_sizes import DECODES, IMAGES, KNOWN, oracle_reduced, u16_sha

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


@pytest.mark.parametrize("which,flags,grok_bytes,grok_sha", KNOWN, ids=[k[1] for k in KNOWN])
def test_engine_equals_grok(eng, images, which, flags, grok_bytes, grok_sha):
    import torch
    img, bits = images[which]
    kw = parse_flags(flags)
    cs = eng.encode(img, bits, params=gk_params(kw))
    assert cs == O.encode(img, bits, **kw), flags
    assert len(cs) == grok_bytes
    if grok_sha:
        assert hashlib.sha256(cs).hexdigest()[:16] == grok_sha
    want, _ = O.decode(cs)
    np.testing.assert_array_equal(eng.decode(cs), want)
    dev = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    np.testing.assert_array_equal(eng.decode(dev, length=len(cs)), want)
    if "-t" in flags:
        h, w = img.shape[1:]
        win = (w // 3, h // 4, w - 5, h - 7)
        np.testing.assert_array_equal(eng.decode_window(dev, win, length=len(cs)), want[:, win[1]:win[3], win[0]:win[2]])


def test_fast_and_serial_simulation_agree(eng, images, monkeypatch):
    # the fast bisection decides a header reaching the budget by coding that packet again through
    # Grok's bounded BitIO; the serial simulation (GK_T2_SERIAL_SIM) runs every step through it
    img, bits = images["A"]
    for flags in ("-t 64,64 -r 40,10 -X -L", "-p CPRL -c [64,64],[32,32] -r 20,5,1", "-t 200,160 -r 30,10"):
        kw = parse_flags(flags)
        fast = eng.encode(img, bits, params=gk_params(kw))
        monkeypatch.setenv("GK_T2_SERIAL_SIM", "1")
        serial = eng.encode(img, bits, params=gk_params(kw))
        monkeypatch.delenv("GK_T2_SERIAL_SIM")
        assert fast == serial, flags


@pytest.mark.parametrize("which,flags,red,win,shape,grok_sha", DECODES, ids=["%s %s -r %d" % (d[0], d[1], d[2]) for d in DECODES])
def test_engine_decode_equals_grok(eng, images, which, flags, red, win, shape, grok_sha):
    # Grok's grk_decompress -r / -d on Grok's own streams (round-5 review hashes): the engine's
    # reduced and windowed decodes equal them and the oracle's
    img, bits = images[which]
    kw = parse_flags(flags)
    cs = eng.encode(img, bits, params=gk_params(kw))
    assert cs == O.encode(img, bits, **kw)
    eng.set_decode_reduce(red)
    try:
        dec = eng.decode_window(cs, win) if win else eng.decode(cs)
    finally:
        eng.set_decode_reduce(0)
    assert dec.shape == shape
    assert u16_sha(dec) == grok_sha
    np.testing.assert_array_equal(dec, oracle_reduced(cs, red, win))
