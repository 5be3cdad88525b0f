"""Components coded with different parameters (main-header COC, with QCC where the quantisation
follows): decomposition levels, code-block size and style (mode switches, HT, wide blocks),
transform and precincts per component (A.6.2; CodeStreamDecompress read_coc / read_SPCod_SPCoc).

The streams are single-component oracle encodes multiplexed into one (tests/coc_mux.py), so the
answer for each component is its own single-component decode.  CPU: the oracle and OpenJPEG 2.5.4
both reproduce it, full and reduced; the engine half is tests/test_gpu_coc.py."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT
import coc_mux
import openjpeg

sys.path.insert(0, os.path.join(ROOT, "oracle"))
import oracle as O  # noqa: E402

# name -> (H, W, prec, per-component oracle.encode keywords, layers)
CASES = {
    "levels_cblk_97_prc": (70, 90, 8, [dict(numres=4), dict(numres=2, cblk=(16, 16)),
                                       dict(numres=3, irreversible=True, precincts=[(32, 32), (16, 16)])], 1),
    "ht_and_part1": (64, 80, 8, [dict(numres=3), dict(numres=3, cblk_sty=0x40), dict(numres=4, cblk=(32, 32))], 1),
    "mode_switches": (60, 72, 8, [dict(numres=3), dict(numres=3, cblk_sty=0x05), dict(numres=2, cblk_sty=0x20)], 1),
    "wide_block": (72, 150, 8, [dict(numres=3), dict(numres=3, cblk=(128, 32))], 1),
    "layers_rate": (96, 96, 8, [dict(numres=4, layer_rate=[20, 5]), dict(numres=3, layer_rate=[30, 8]),
                                dict(numres=5, irreversible=True, layer_rate=[40, 10])], 2),
    "mono12_pair": (50, 66, 12, [dict(numres=5, cblk=(32, 32)), dict(numres=1)], 1),
    # components of different precisions (SIZ Ssiz per component; QCC follows the precision)
    "mixed_precision": (48, 60, [12, 8, 16, 4], [dict(numres=3), dict(numres=3), dict(numres=4, irreversible=True),
                                                 dict(numres=2)], 1),
}


def _precs(name):
    H, W, prec, kws, L = CASES[name]
    return list(prec) if isinstance(prec, (list, tuple)) else [prec] * len(kws)


def planes(name):
    H, W, prec, kws, L = CASES[name]
    rng = np.random.default_rng(sum(map(ord, name)))
    yy, xx = np.mgrid[0:H, 0:W]
    return [((xx * (c + 2) + yy * 3 + rng.integers(0, 16, size=(H, W))) % (1 << pr)).astype(np.int32)
            for c, pr in enumerate(_precs(name))]


def stream(name):
    H, W, prec, kws, L = CASES[name]
    return coc_mux.mux(planes(name), prec, kws, nlayers=L)


def single_decodes(name, reduce=0):
    """Each component's own single-component stream, decoded by the oracle."""
    H, W, prec, kws, L = CASES[name]
    out = []
    O.set_decode_reduce(reduce)
    try:
        for p, kw, pr in zip(planes(name), kws, _precs(name)):
            kw = dict(kw, plt=True, mct=False, write_com=False)
            if "layer_rate" not in kw:
                kw["nlayers"] = L
            out.append(O.decode(O.encode(p[None], pr, **kw))[0][0])
    finally:
        O.set_decode_reduce(0)
    return out


@pytest.mark.parametrize("name", sorted(CASES))
def test_oracle_coc_equals_single_component_decodes(name):
    got, _ = O.decode(stream(name))
    for g, w in zip(got, single_decodes(name)):
        np.testing.assert_array_equal(g, w)


@pytest.mark.skipif(not openjpeg.available(), reason="libopenjp2 (Pillow's) not present")
@pytest.mark.parametrize("name", sorted(CASES))
def test_openjpeg_coc_equals_single_component_decodes(name):
    ref = openjpeg.decode(stream(name))
    for (dx, dy, r), w in zip(ref, single_decodes(name)):
        np.testing.assert_array_equal(r, w)


@pytest.mark.parametrize("name", ["levels_cblk_97_prc", "ht_and_part1", "layers_rate"])
def test_oracle_coc_reduced(name):
    cs = stream(name)
    O.set_decode_reduce(1)
    try:
        got, _ = O.decode(cs)
    finally:
        O.set_decode_reduce(0)
    for g, w in zip(got, single_decodes(name, reduce=1)):
        np.testing.assert_array_equal(g, w)


def test_mixed_precision_reported():
    O.decode(stream("mixed_precision"))
    assert O.last_comp_prec() == [(12, False), (8, False), (16, False), (4, False)]
    import grok_amd as G
    assert [c[2] for c in G.probe_components(stream("mixed_precision"), precision=True)] == [12, 8, 16, 4]
    assert G.probe_header(stream("mixed_precision")).prec == 16   # (the largest)


def test_oracle_coc_reduce_past_a_component_refused():
    # mono12_pair's second component has a single resolution: reduce 1 leaves it none
    O.set_decode_reduce(1)
    try:
        with pytest.raises(RuntimeError, match="-7"):
            O.decode(stream("mono12_pair"))
    finally:
        O.set_decode_reduce(0)
