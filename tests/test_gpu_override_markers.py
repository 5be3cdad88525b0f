"""COC / QCC and tile-part COD / QCD markers in the HIP decoder (the oracle half and the
rationale are in tests/test_override_markers.py): markers restating the main COD / QCD decode
exactly as the stream without them, from host and from device-resident (TLM-located) streams;
markers that change a tile's coding decode to the oracle's samples; bad component numbers are
refused with the engine's message."""
import numpy as np
import pytest

from conftest import FIXTURES
from test_override_markers import NAMES, changing, refused, restating

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


def _fx(name):
    return next(f for f in FIXTURES if f.name == name)


@pytest.mark.parametrize("name", NAMES)
def test_restating_markers_engine(eng, name):
    import torch
    fx = _fx(name)
    cs = restating(fx.cs)
    np.testing.assert_array_equal(eng.decode(cs), fx.grok_decoded)
    d = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    np.testing.assert_array_equal(eng.decode(d, len(cs)), fx.grok_decoded)


@pytest.mark.parametrize("name", NAMES)
def test_changing_tile_markers_engine(eng, name):
    import oracle as O
    import torch
    fx = _fx(name)
    for what, cs in changing(fx.cs):
        if fx.ht and what == "tile COC":
            with pytest.raises(RuntimeError, match="HTJ2K combined with Part-1"):
                eng.decode(cs)
            continue
        want = O.decode(cs)[0]
        np.testing.assert_array_equal(eng.decode(cs), want, err_msg=what)
        d = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
        np.testing.assert_array_equal(eng.decode(d, len(cs)), want, err_msg=what)
    for what, cs in refused(fx.cs):
        with pytest.raises(RuntimeError, match="bad component number"):
            eng.decode(cs)
    np.testing.assert_array_equal(eng.decode(fx.cs), fx.grok_decoded)


@pytest.mark.parametrize("name", NAMES)
def test_main_qcc_engine_equals_oracle(eng, name):
    import j2k_markers as J
    import oracle as O
    fx = _fx(name)
    cs = J.insert_main(fx.cs, J.qcc(fx.cs, J.ncomp(fx.cs) - 1, guard_add=1))
    np.testing.assert_array_equal(eng.decode(cs), O.decode(cs)[0])
