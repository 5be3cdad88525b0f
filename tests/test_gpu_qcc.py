"""The HIP decoder on per-component (QCC) and scalar-derived quantisation (tests/qcc_cases.py;
the oracle's decode of these streams is pinned by OpenJPEG 2.5.4 in tests/test_qcc.py): whole
image from host and device memory, and a window, sample-equal to the oracle."""
import numpy as np
import pytest

import oracle as O
from qcc_cases import CASES

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


@pytest.mark.parametrize("name,shape,bits,kw", CASES, ids=[c[0] for c in CASES])
def test_qcc_decode_vs_oracle(eng, name, shape, bits, kw):
    import torch
    from grok_amd.synth import synth_image
    c, h, w = shape
    img = synth_image(h, w, c, bits, 61).astype(np.int32)
    cs = O.encode(img, bits, **kw)
    want, _ = O.decode(cs)
    np.testing.assert_array_equal(eng.decode(cs), want)
    d = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    np.testing.assert_array_equal(eng.decode(d, length=len(cs)), want)
    win = (w // 4, h // 5, w - 3, h - 7)
    np.testing.assert_array_equal(eng.decode_window(cs, win),
                                  O.decode(cs, partial=True)[0][:, win[1]:win[3], win[0]:win[2]])
    # the engine's own encode of the same image (one QCD, Grok's) still decodes after the QCC stream
    import grok_amd as G
    k = {kk: v for kk, v in kw.items() if kk not in ("comp_guard_bits", "comp_qshift", "qderived")}
    if "numres" in k:
        k["numresolution"] = k.pop("numres")
    if "layer_rate" in k:
        k["numlayers"] = len(k["layer_rate"])
    own = eng.encode(img, bits, params=G.default_params(**k))
    np.testing.assert_array_equal(eng.decode(own), O.decode(own)[0])
