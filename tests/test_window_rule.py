"""The oracle's two inverse 5/3 rules on a stream where they differ (tests/window_rule_case.py):
the engine's grk_decompress_tile without a window must take the whole-tile one, a window the
partial-tile one (tests/test_gpu_grk_api.py)."""
import numpy as np

import oracle as O
from window_rule_case import LAYERS, case


def test_rules_differ_on_fixture():
    img, kw = case()
    cs = O.encode(img, 8, **kw)
    O.set_decode_layers(LAYERS)
    try:
        whole, _ = O.decode(cs)
        part, _ = O.decode(cs, partial=True)
    finally:
        O.set_decode_layers(0)
    diff = np.nonzero((whole != part)[0])
    assert len(diff[0]) > 0
    assert diff[1].min() >= 36 and diff[1].max() < 48      # inside tile 3 only


def test_single_sample_rules():
    # WaveletReverse.cpp:583 bandH[0] / 2 (toward zero) vs :1551-1554 >>= 1 (toward -inf)
    lib = O.lib()
    assert lib.orc_inv53_single(-7, 1, 0, 0) == -3
    assert lib.orc_inv53_single(-7, 1, 0, 1) == -4
    assert lib.orc_inv53_single(7, 1, 0, 0) == lib.orc_inv53_single(7, 1, 0, 1) == 3
