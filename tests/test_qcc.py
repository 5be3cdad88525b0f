"""Per-component (QCC) and scalar-derived quantisation in the oracle (tests/qcc_cases.py).

Oracle encode -> oracle decode round trips (lossless for 5/3), and the decode is pinned by an
independent decoder: OpenJPEG 2.5.4 through Pillow decodes the same streams to the same samples
(5/3 and 9/7).  Grok has no reference output for them (its encoder never writes QCC or derived
steps): parity with Grok itself is unpinned, its decoder's rules are restated from
Quantizer::read_SQcd_SQcc (Quantizer.cpp:185-334) and checked by the derived-step expansion test."""
import io

import numpy as np
import pytest

import oracle as O
from qcc_cases import CASES


def _img(shape, bits, seed):
    from grok_amd.synth import synth_image
    c, h, w = shape
    return synth_image(h, w, c, bits, seed).astype(np.int32)


def _markers(cs):
    """(marker, body) of the main header, SOC to the first SOT."""
    i, out = 2, []
    while i + 4 <= len(cs):
        m = int.from_bytes(cs[i:i + 2], "big")
        if m == 0xFF90:
            break
        L = int.from_bytes(cs[i + 2:i + 4], "big")
        out.append((m, cs[i + 4:i + 2 + L]))
        i += 2 + L
    return out


@pytest.mark.parametrize("name,shape,bits,kw", CASES, ids=[c[0] for c in CASES])
def test_qcc_round_trip_and_openjpeg(name, shape, bits, kw):
    from PIL import Image
    img = _img(shape, bits, 61)
    cs = O.encode(img, bits, **kw)
    mk = _markers(cs)
    nq = sum(1 for m, _ in mk if m == 0xFF5D)
    want_q = 0 if name == "irr_derived" else sum(1 for c in range(1, shape[0])
                                                  if (kw.get("comp_guard_bits") or [2] * 3)[c] != (kw.get("comp_guard_bits") or [2] * 3)[0]
                                                  or (kw.get("comp_qshift") or [0] * 3)[c] != (kw.get("comp_qshift") or [0] * 3)[0])
    assert nq == want_q
    if kw.get("qderived"):
        qcd = next(b for m, b in mk if m == 0xFF5C)
        assert qcd[0] & 0x1F == 1 and len(qcd) == 3        # Sqcd style 1: the LL step only
    dec, _ = O.decode(cs)
    if not kw.get("irreversible") and not kw.get("layer_rate"):
        np.testing.assert_array_equal(dec, img)
    else:
        mse = ((dec.astype(np.float64) - img) ** 2).mean()
        assert 10 * np.log10(((1 << bits) - 1) ** 2 / mse) > 28
    if bits == 8 or shape[0] == 1:
        a = np.asarray(Image.open(io.BytesIO(cs))).astype(np.int32)
        a = a.transpose(2, 0, 1) if a.ndim == 3 else a[None]
        np.testing.assert_array_equal(a, dec)


def test_derived_steps_follow_e5():
    # Sqcd style 1 with epsilon_0 = 20, mu_0 = 77 at 6 resolutions: band b > 0 at resolution r
    # (b = 3 (r - 1) + 1 ..) takes epsilon_0 - (r - 1) (Quantizer.cpp:319-331; E-5 epsilon_0 - N_L +
    # n_b with n_b = N_L - r + 1); re-encoding those steps expounded gives the same decode
    img = _img((3, 128, 128), 8, 5)
    a = O.encode(img, 8, irreversible=True, qderived=True)
    qcd = next(b for m, b in _markers(a) if m == 0xFF5C)
    e0, m0 = qcd[1] >> 3, ((qcd[1] & 7) << 8) | qcd[2]
    exp = [(e0, m0)] + [(e0 - (r - 1), m0) for r in range(1, 6) for _ in range(3)]
    # the same image coded expounded with those exact steps (QCD rewritten, T1 data unchanged) decodes alike
    body = bytes([qcd[0] & 0xE0 | 2]) + b"".join(((e << 11) | m).to_bytes(2, "big") for e, m in exp)
    i = a.index(b"\xff\x5c")
    L = int.from_bytes(a[i + 2:i + 4], "big")
    b = a[:i] + b"\xff\x5c" + (2 + len(body)).to_bytes(2, "big") + body + a[i + 2 + L:]
    np.testing.assert_array_equal(O.decode(a)[0], O.decode(b)[0])
