"""Caller COM markers (grk_cparameters comment / comment_len / is_binary_comment / num_comments,
grk_compress -C; CodeStreamCompress.cpp:303-330, write_com :1114-1145): written instead of Grok's
default comment, text (Rcom 1) or binary (Rcom 0); with rate control their bytes count in the
header size updateRates spreads over the tiles.  The engine writes the oracle's bytes."""
import numpy as np
import pytest

import oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("kw", [dict(numres=4), dict(numres=5, layer_rate=[30, 8]), dict(numres=3, tiles=(64, 48), layer_rate=[20])])
def test_engine_comments_equal_oracle(kw):
    import grok_amd as G
    from grok_amd.synth import synth_image
    img = synth_image(100, 130, 3, 8, 17).astype(np.int32)
    comments = ["made by a test", b"\x00\xffbinary\x01"]
    e = G.Engine(0)
    try:
        gk = dict(kw)
        gk["numresolution"] = gk.pop("numres")
        cs = e.encode(img, 8, params=G.default_params(mct=True, comments=comments, **gk))
    finally:
        e.close()
    assert cs == O.encode(img, 8, comments=comments, **kw)
    head = cs[:cs.index(b"\xff\x90")]   # (the main header: packet data may hold FF64 too)
    assert head.count(b"\xff\x64") == 2 and b"Created by Grok" not in head
