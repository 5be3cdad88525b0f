"""SOP / EPH markers (grk_compress -S / -E: csty bits 2 / 4, T2Compress.cpp:286-320 and
T2Decompress.cpp:226-250, 469-486) and fixed-quality layers (grk_compress -q,
allocationByQuality: TileProcessor.cpp:1263-1322) on the HIP path vs the oracle.

Encode: byte-identical codestreams (SOP counters per tile, EPH after every header, PLT lengths
that include them; under rate control the T2 simulation takes SOP's 6 and EPH's 2 bytes in
Grok's uint32 arithmetic; under -q the bisection compares the layer's distortion with the PSNR
target instead of simulating).  Decode: the engine reads the oracle's streams sample-exactly.
Parity unpinned against Grok itself (no Grok-made SOP/EPH or -q stream is held here)."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


def _img(seed, c, h, w, bits):
    from grok_amd.synth import synth_image
    return synth_image(h, w, c, bits, seed).astype(np.int32)


def _gk(kw):
    import grok_amd as G
    kw = dict(kw)
    if "numres" in kw:
        kw["numresolution"] = kw.pop("numres")
    if "layer_rate" in kw:
        kw["numlayers"] = len(kw["layer_rate"])
    return G.default_params(**kw)


CASES = [
    ("sop", 3, 200, 300, 8, dict(sop=True)),
    ("eph", 3, 200, 300, 8, dict(eph=True)),
    ("sop_eph", 3, 200, 300, 8, dict(sop=True, eph=True)),
    ("sop_eph_r", 3, 256, 256, 8, dict(sop=True, eph=True, layer_rate=[20.0, 5.0])),
    ("sop_eph_97_r", 3, 256, 320, 12, dict(sop=True, eph=True, irreversible=True, layer_rate=[40.0, 20.0, 10.0])),
    ("sop_eph_tiles", 3, 300, 260, 8, dict(sop=True, eph=True, tiles=(128, 128), plt=True, tlm=True, layer_rate=[10.0])),
    ("sop_rpcl_prc", 3, 192, 256, 8, dict(sop=True, eph=True, prog_order="RPCL", precincts=[(64, 64)])),
    ("sop_eph_ht", 1, 256, 256, 16, dict(sop=True, eph=True, cblk_sty=0x40, tiles=(128, 128), tlm=True, plt=True)),
    ("sop_tp_r", 3, 256, 256, 8, dict(sop=True, eph=True, tile_parts="R", tiles=(128, 128))),
    ("q30_40", 3, 256, 256, 8, dict(quality=[30.0, 40.0])),
    ("q28_36_0", 3, 200, 300, 8, dict(quality=[28.0, 36.0, 0.0])),
    ("q35_97", 3, 256, 320, 12, dict(quality=[35.0, 42.0], irreversible=True)),
    ("q_tiles", 3, 300, 260, 8, dict(quality=[30.0, 38.0], tiles=(128, 128), tlm=True)),
    ("q_sop_eph", 1, 256, 256, 16, dict(quality=[45.0, 60.0], sop=True, eph=True)),
]


@pytest.mark.parametrize("case", CASES, ids=[c[0] for c in CASES])
def test_encode_decode_vs_oracle(eng, case):
    name, c, h, w, bits, kw = case
    img = _img(70 + len(name), c, h, w, bits)
    ref = O.encode(img, bits, **kw)
    cs = eng.encode(img, bits, params=_gk(kw))
    assert cs == ref
    want, _ = O.decode(ref)
    np.testing.assert_array_equal(eng.decode(ref), want)
    if "layer_rate" not in kw and "quality" not in kw:
        np.testing.assert_array_equal(want, img)
    if "quality" in kw and kw["quality"][-1] == 0:
        np.testing.assert_array_equal(want, img)


def test_sop_window_decode(eng):
    # PLT-guided window decode skips packets whose SOP / EPH bytes are counted in the PLT lengths
    img = _img(5, 3, 384, 384, 8)
    kw = dict(sop=True, eph=True, tiles=(128, 128), tlm=True, plt=True)
    cs = O.encode(img, 8, **kw)
    np.testing.assert_array_equal(eng.decode_window(cs, (37, 50, 301, 350)), img[:, 50:350, 37:301])
