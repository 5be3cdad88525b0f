"""Tile sharding across ranks on CPU (gloo, world size 2): the distributed
plumbing of grok_amd/shard.py — tile-row split, length + payload gather, TLM
fill, tile-part ordering, per-rank partial decode — with the oracle standing in
for the per-rank GPU coder (each rank's tile parts are cut from the oracle's
full-image codestream; decode of header + a subset of tile parts is the oracle's
decoder).  The assembled codestream must equal the one-process encode byte for
byte, and the gathered decode must equal the source.  The GPU path runs the
same functions with gk_encode_tiles / gk_decode (tests/test_gpu_tiles.py).
"""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

import oracle as O
from grok_amd import shard

CASES = [
    dict(shape=(1, 300, 200), bits=16, kw=dict(tiles=(64, 64), cblk_sty=64, tlm=True, plt=True)),
    dict(shape=(3, 257, 130), bits=8, kw=dict(tiles=(64, 32), numres=4, tlm=True)),
    dict(shape=(1, 100, 100), bits=8, kw=dict(tiles=(128, 128))),   # one tile: rank 1 idle
]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, case, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        c, h, w = case["shape"]
        rng = np.random.default_rng(1)
        img = rng.integers(0, 1 << case["bits"], size=(c, h, w)).astype(np.int32)
        kw = case["kw"]
        tw, th = kw["tiles"]
        ntx, nty = shard.tile_grid(h, w, th, tw)
        full = O.encode(img, case["bits"], **kw)
        header, parts = shard.split_codestream(full)
        pmap = dict(parts)

        def encode_tiles(tb, te):   # stand-in for gk_encode_tiles on this rank's device
            blob = b"".join(pmap[t] for t in range(tb, te))
            return blob, [len(pmap[t]) for t in range(tb, te)]

        def main_header():
            tlm = 0
            if kw.get("tlm"):
                i = header.index(b"\xff\x55")
                tlm = i + 6
            return header, tlm

        cs = shard.encode_sharded(dist, rank, world, encode_tiles, main_header, ntx, nty)

        def dec_rows(sub, y0, y1):   # stand-in for gk_decode of the rank's sub-stream into its slab
            d, _ = O.decode(sub.numpy().tobytes())
            return d[:, y0:y1]

        dec = shard.decode_sharded(dist, rank, world, full if rank == 0 else None, dec_rows, ntx, nty, th, (c, h, w))
        if rank == 0:
            q.put((cs == full, bool((dec.numpy() == img).all())))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("case", CASES, ids=["ht16_tlm_plt", "rgb8_tlm", "single_tile"])
def test_sharded_encode_decode_gloo(case):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, case, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == (True, True)


def test_rank_tiles_cover_grid():
    for ntx, nty, world in [(16, 16, 8), (3, 5, 2), (1, 1, 4), (4, 3, 8)]:
        seen = []
        for r in range(world):
            tb, te, j0, j1 = shard.rank_tiles(ntx, nty, r, world)
            assert te - tb == (j1 - j0) * ntx
            seen += list(range(tb, te))
        assert seen == list(range(ntx * nty))


def test_retlm_lists_only_given_parts():
    rng = np.random.default_rng(4)
    img = rng.integers(0, 256, size=(1, 96, 160)).astype(np.int32)
    cs = O.encode(img, 8, tiles=(32, 32), tlm=True, plt=True)
    header, parts = shard.split_codestream(cs)
    mine = parts[5:10]
    sub = shard.retlm(header, [(t, len(b)) for t, b in mine]) + b"".join(b for _, b in mine) + b"\xff\xd9"
    d, _ = O.decode(sub)
    np.testing.assert_array_equal(d[:, 32:64], img[:, 32:64])
    i = sub.index(b"\xff\x55")
    assert int.from_bytes(sub[i + 2:i + 4], "big") == 4 + 6 * 5
    plain = shard.split_codestream(O.encode(img, 8, tiles=(32, 32)))[0]   # no TLM: header unchanged
    assert shard.retlm(plain, [(0, 10)]) == plain


def test_assemble_roundtrip():
    rng = np.random.default_rng(3)
    img = rng.integers(0, 256, size=(1, 96, 160)).astype(np.int32)
    cs = O.encode(img, 8, tiles=(32, 32), tlm=True, plt=True)
    header, parts = shard.split_codestream(cs)
    assert [t for t, _ in parts] == list(range(15))
    # zero the TLM entries and rebuild them from the parts
    i = header.index(b"\xff\x55")
    h = bytearray(header)
    h[i + 6:i + 6 + 6 * 15] = bytes(90)
    assert shard.assemble(bytes(h), i + 6, parts[::-1]) == cs
