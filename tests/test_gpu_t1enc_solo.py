"""Solo MQ encode waves (gk_t1enc.hip mq_solo_block): the heaviest code-blocks coded one per wave
with the coder wave-uniform.  Every split of the blocks between solo and lane-parallel waves must
give the oracle's codestream byte for byte (GK_T1ENC_SOLO = the number of blocks on solo waves:
without chunks the first blocks in index order, with chunks the heaviest of the first chunk),
with and without rate control (pass rates and distortions feed PCRD)."""
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


def _params(kw):
    import grok_amd as G
    k = dict(kw)
    if "layer_rate" in k:
        k["numlayers"] = len(k["layer_rate"])
    if "numres" in k:
        k["numresolution"] = k.pop("numres")
    return G.default_params(**k)


CASES = [
    ("rgb8", (3, 300, 420), 8, {}),
    ("rgb12_97_rc", (3, 260, 300), 12, dict(irreversible=True, layer_rate=[40.0, 20.0, 10.0])),
    ("mono16_rc", (1, 333, 257), 16, dict(layer_rate=[30.0, 8.0], cblk=(32, 32))),
    ("rgb8_tiles", (3, 200, 310), 8, dict(tiles=(128, 96), numres=4)),
]


@pytest.mark.parametrize("nsolo", [1, 7, 64, 100000])
@pytest.mark.parametrize("name,shape,bits,kw", CASES, ids=[c[0] for c in CASES])
def test_solo_split_vs_oracle(eng, monkeypatch, name, shape, bits, kw, nsolo):
    from grok_amd.synth import synth_image
    c, h, w = shape
    img = synth_image(h, w, c, bits, 90 + nsolo % 7).astype(np.int32)
    ref = O.encode(img, bits, **kw)
    monkeypatch.setenv("GK_T1ENC_SOLO", str(nsolo))
    cs = eng.encode(img, bits, params=_params(kw))
    assert cs == ref, (name, nsolo, len(cs), len(ref))


def test_solo_chunked_large(eng, monkeypatch):
    # >= 8192 blocks: the chunked modelling / MQ overlap, solo waves in the first (heaviest) chunk
    from grok_amd.synth import synth_image
    img = synth_image(2048, 2048, 3, 12, 11).astype(np.int32)   # 12,288 blocks of 32 x 32
    kw = dict(irreversible=True, layer_rate=[40.0, 20.0, 10.0], cblk=(32, 32))
    ref = O.encode(img, 12, **kw)
    for nsolo in (0, 48, 256):
        monkeypatch.setenv("GK_T1ENC_SOLO", str(nsolo))
        assert eng.encode(img, 12, params=_params(kw)) == ref, nsolo
