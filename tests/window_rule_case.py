"""A stream whose tile decode depends on the inverse 5/3 rule.

Tiles 12 samples wide with 5 resolutions leave one-sample-wide resolutions on odd canvas
coordinates; signed 8-bit noise coded in 7 rate-controlled layers and decoded with 6 of them
leaves odd negative high-pass samples there.  Grok halves such a sample in the whole-tile inverse
(WaveletReverse.cpp:583, decompressTile without a window) and shifts it in the partial-tile one
(:1551-1554, any decode after setDecompressWindow), so the two decodes differ."""
import numpy as np

LAYERS = 6
TILE = 3   # the tile at canvas x 36..48: the rules differ there


def case():
    rng = np.random.default_rng(243)
    h = int(rng.integers(64, 200))
    w = int(rng.integers(30, 90))
    tw = int(rng.choice([3, 6, 12, 24]))
    assert tw == 12
    img = (rng.integers(-128, 128, size=(1, h, w)) * rng.random((1, h, w))).astype(np.int32)
    kw = dict(signed=True, tiles=(tw, h), numres=5, layer_rate=[60, 30, 15, 8, 5, 3, 2])
    return img, kw
