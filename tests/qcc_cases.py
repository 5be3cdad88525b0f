"""Streams with per-component quantisation (QCC, A.6.5) and scalar-derived quantisation (Sqcd
style 1, E-5), as third-party encoders write them (Grok's own encoder pushes one QCD to every
component, CodeStreamCompress.cpp:382-384, and writes expounded steps).  The oracle writes them
(oracle.params comp_guard_bits / comp_qshift / qderived); OpenJPEG 2.5.4 (Pillow), an
independent decoder, pins their decode (tests/test_qcc.py)."""
CASES = [
    ("rev_gb", (3, 200, 240), 8, dict(comp_guard_bits=[2, 1, 3])),
    ("rev_gb_mono16", (1, 150, 170), 16, dict(comp_guard_bits=[3])),
    ("irr_qshift", (3, 200, 240), 8, dict(irreversible=True, comp_qshift=[0, 1, 2])),
    ("irr_derived", (3, 180, 210), 12, dict(irreversible=True, qderived=True)),
    ("irr_derived_qcc", (3, 200, 240), 8, dict(irreversible=True, qderived=True, comp_qshift=[0, 2, 1],
                                                comp_guard_bits=[2, 2, 1])),
    ("irr_nomct_qcc_tiles", (3, 170, 230), 8, dict(irreversible=True, mct=False, comp_qshift=[1, 0, 2],
                                                    tiles=(64, 80), layer_rate=[30.0, 10.0])),
    ("rev_gb_prc_tiles", (3, 190, 201), 8, dict(comp_guard_bits=[1, 2, 2], tiles=(96, 64),
                                                 precincts=[(32, 32)], numres=4)),
]
