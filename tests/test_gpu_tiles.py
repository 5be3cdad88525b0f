"""Multi-tile images on the HIP path (batched per-tile DWT, all tiles' code-blocks
in one T1 launch, per-tile T2, SOT/TLM/PLT) vs Grok and the oracle.

Bar: codestreams byte-identical to
Grok's `-t W,H [-X] [-L]` output (fixtures) and to the oracle on seeded random
tilings (ragged edge tiles, 1-tile-wide strips, Part 1 and HT, TLM/PLT on and
off); decodes sample-exact.  These tilings are multiples of 2^(levels) (tile DWT parity 0,
the C4/C5 configurations); other tile sizes are tests/test_gpu_odd_tiles.py.
"""
import numpy as np
import pytest

from conftest import FIXTURES, ROOT, fixture_ids
import oracle as O

pytestmark = pytest.mark.gpu

TILED = [f for f in FIXTURES if f.tiled]


@pytest.fixture(scope="module")
def eng():
    import grok_amd as G
    e = G.Engine(0)
    yield e
    e.close()


def _params(**kw):
    import grok_amd as G
    numres = kw.pop("numres", 6)
    return G.default_params(numresolution=numres, **kw)


@pytest.mark.parametrize("fx", TILED, ids=fixture_ids(TILED))
def test_tiled_fixture_encode_bit_exact(eng, fx):
    from test_gpu_parity import gk_params
    cs = eng.encode(fx.img, fx.bits, params=gk_params(fx.kw))
    assert cs == fx.cs


@pytest.mark.parametrize("fx", TILED, ids=fixture_ids(TILED))
def test_tiled_fixture_decode(eng, fx):
    dec = eng.decode(fx.cs)
    if fx.lossless:
        np.testing.assert_array_equal(dec, fx.img)
    else:
        assert np.abs(dec.astype(np.int64) - fx.grok_decoded).max() <= 1


@pytest.mark.parametrize("seed", range(16))
def test_tiled_random_vs_oracle(eng, seed):
    rng = np.random.default_rng(700 + seed)
    numres = int(rng.integers(1, 7))
    unit = 1 << (numres - 1)
    tw = unit * int(rng.integers(1, max(2, 256 // unit) + 1))
    th = unit * int(rng.integers(1, max(2, 256 // unit) + 1))
    w, h = int(rng.integers(1, 3 * tw + 5)), int(rng.integers(1, 3 * th + 5))
    c = int(rng.choice([1, 3]))
    bits = int(rng.choice([8, 12, 16]))
    ht = bool(seed % 2)
    tlm, plt = bool(seed % 3 == 0), bool(seed % 4 < 2)
    cb = [(64, 64), (32, 32), (16, 64)][seed % 3]
    img = rng.integers(0, 1 << bits, size=(c, h, w)).astype(np.int32)
    kw = dict(numres=numres, cblk=cb, tiles=(tw, th), tlm=tlm, plt=plt, cblk_sty=64 if ht else 0)
    ref = O.encode(img, bits, **kw)
    gkw = dict(kw)
    gkw["numres"] = gkw["numres"]
    cs = eng.encode(img, bits, params=_params(**gkw))
    assert cs == ref, (w, h, tw, th, numres, ht)
    np.testing.assert_array_equal(eng.decode(cs), img)
    # device-resident codestream: TLM-located tile parts, PLT-batched packet headers
    import torch
    d = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    y = torch.empty((c, h, w), dtype=torch.int32, device="cuda")
    eng.decode(d, length=len(cs), out=y)
    np.testing.assert_array_equal(y.cpu().numpy(), img)


def test_tiled_97(eng):
    rng = np.random.default_rng(5)
    img = rng.integers(0, 4096, size=(3, 200, 260)).astype(np.int32)
    kw = dict(tiles=(128, 64), irreversible=True, tlm=True, plt=True)
    ref = O.encode(img, 12, **kw)
    cs = eng.encode(img, 12, params=_params(**kw))
    assert cs == ref
    dec_o, _ = O.decode(cs)
    assert np.abs(eng.decode(cs).astype(np.int64) - dec_o).max() <= 1


def test_tile_grid_rules(eng):
    # tile sizes off the 2^levels grid: odd-parity levels (tests/test_gpu_odd_tiles.py)
    img = (np.arange(100 * 100, dtype=np.int32).reshape(1, 100, 100) * 7) % 251
    cs = eng.encode(img, 8, params=_params(tiles=(48, 48)))
    assert cs == O.encode(img, 8, tiles=(48, 48))
    np.testing.assert_array_equal(eng.decode(cs), img)
    # a tile larger than the image is a single tile
    cs = eng.encode(img, 8, params=_params(tiles=(4096, 4096)))
    np.testing.assert_array_equal(eng.decode(cs), img)


def test_engine_reuse_refreshes_params(eng):
    # same geometry, different non-geometric parameters (TLM/PLT, layer rates): the
    # cached plan must not carry the previous call's settings over
    rng = np.random.default_rng(77)
    img = rng.integers(0, 256, size=(3, 256, 256)).astype(np.int32)
    for kw in (dict(tiles=(128, 128)), dict(tiles=(128, 128), tlm=True, plt=True), dict(tiles=(128, 128))):
        assert eng.encode(img, 8, params=_params(**kw)) == O.encode(img, 8, **kw)
    for rates in ([40.0, 20.0], [20.0, 10.0], [40.0, 20.0]):
        kw = dict(irreversible=True, layer_rate=rates)
        assert eng.encode(img, 8, params=_params(**kw)) == O.encode(img, 8, **kw)


def _c4_like(seed=3):
    rng = np.random.default_rng(seed)
    return rng.integers(0, 1 << 16, size=(1, 320, 288)).astype(np.int32)


@pytest.mark.parametrize("world", [2, 3])
def test_encode_tiles_assemble_equals_full(eng, world):
    # each "rank" encodes its tile rows from its own slab; header + parts == one-shot encode
    from grok_amd import shard
    img = _c4_like()
    kw = dict(tiles=(64, 64), cblk_sty=64, tlm=True, plt=True)
    full = eng.encode(img, 16, params=_params(**kw))
    assert full == O.encode(img, 16, **kw)
    _, h, w = img.shape
    ntx, nty = shard.tile_grid(h, w, 64, 64)
    parts = []
    for r in range(world):
        tb, te, j0, j1 = shard.rank_tiles(ntx, nty, r, world)
        y0, y1 = j0 * 64, min(h, j1 * 64)
        blob, lens = eng.encode_tiles(img[:, y0:y1], 16, tb, te, image_hw=(h, w), row0=y0, params=_params(**kw))
        parts += shard.split_parts(blob, lens, tb)
    header, tlm, nt = eng.main_header(img.shape, 16, params=_params(**kw))
    assert nt == ntx * nty
    assert shard.assemble(header, tlm, parts) == full


def test_decode_subset_of_tiles(eng):
    from grok_amd import shard
    img = _c4_like(4)
    kw = dict(tiles=(64, 64), tlm=True)
    cs = eng.encode(img, 16, params=_params(**kw))
    header, parts = shard.split_codestream(cs)
    ntx = (img.shape[2] + 63) // 64
    sub = header + b"".join(b for t, b in parts if 2 * ntx <= t < 4 * ntx) + b"\xff\xd9"
    dec = eng.decode(sub)
    np.testing.assert_array_equal(dec[:, 128:256], img[:, 128:256])


def _gpu_shard_worker(rank, world, port, q):
    import os
    import torch
    import torch.distributed as dist
    import grok_amd as G
    from grok_amd import shard
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)   # two ranks share the one GPU
    try:
        e = G.Engine(0)
        img = _c4_like(5)
        _, h, w = img.shape
        kw = dict(tiles=(64, 64), cblk_sty=64, tlm=True, plt=True)
        p = G.default_params(**kw)
        ntx, nty = shard.tile_grid(h, w, 64, 64)

        def enc(tb, te):
            j0, j1 = tb // ntx, te // ntx
            y0, y1 = j0 * 64, min(h, j1 * 64)
            return e.encode_tiles(img[:, y0:y1], 16, tb, te, image_hw=(h, w), row0=y0, params=p)

        def hdr():
            hd, tlm, _ = e.main_header(img.shape, 16, params=p)
            return hd, tlm

        cs = shard.encode_sharded(dist, rank, world, enc, hdr, ntx, nty)
        def dec_rows(sub, y0, y1):   # the rank's sub-stream (header with its own TLM + parts) into its slab
            d = sub.cuda()
            out = torch.empty((img.shape[0], y1 - y0, w), dtype=torch.int32, device="cuda")
            e.decode(d, length=d.numel(), out=out, row0=y0)
            return out.cpu()

        dec = shard.decode_sharded(dist, rank, world, cs, dec_rows, ntx, nty, 64, img.shape)
        dec = dec.numpy() if dec is not None else None
        if rank == 0:
            q.put((cs == O.encode(img, 16, **kw), bool((dec == img).all())))
        e.close()
    finally:
        dist.destroy_process_group()


def test_sharded_two_processes_one_gpu():
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_gpu_shard_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == (True, True)


@pytest.mark.parametrize("seed", range(8))
def test_decode_window_vs_full(eng, seed):
    # random windows (aligned, unaligned, edge, whole image) of tiled Part-1 / HT / 9/7
    # streams, host and device codestreams: window decode == crop of the full decode
    import torch
    rng = np.random.default_rng(900 + seed)
    c = int(rng.choice([1, 3]))
    bits = 8 if c == 3 else 16
    h, w = int(rng.integers(64, 400)), int(rng.integers(64, 400))
    img = rng.integers(0, 1 << bits, size=(c, h, w)).astype(np.int32)
    kind = seed % 3
    kw = dict(tiles=(64, 64), tlm=bool(seed % 2), plt=bool(seed % 2), numres=4)
    if kind == 1:
        kw["cblk_sty"] = 64
    if kind == 2:
        kw["irreversible"] = True
    cs = eng.encode(img, bits, params=_params(**kw))
    full = eng.decode(cs)
    if kind != 2:
        np.testing.assert_array_equal(full, img)
    d = torch.frombuffer(bytearray(cs), dtype=torch.uint8).cuda()
    for _ in range(4):
        x0, y0 = int(rng.integers(0, w)), int(rng.integers(0, h))
        x1, y1 = int(rng.integers(x0 + 1, w + 1)), int(rng.integers(y0 + 1, h + 1))
        np.testing.assert_array_equal(eng.decode_window(cs, (x0, y0, x1, y1)), full[:, y0:y1, x0:x1])
        y = torch.empty((c, y1 - y0, x1 - x0), dtype=torch.int32, device="cuda")
        eng.decode_window(d, (x0, y0, x1, y1), length=len(cs), out=y)
        np.testing.assert_array_equal(y.cpu().numpy(), full[:, y0:y1, x0:x1])
    np.testing.assert_array_equal(eng.decode_window(cs, (0, 0, w, h)), full)


def test_decode_window_single_tile(eng):
    fx = [f for f in FIXTURES if f.name == "rgb8_odd"][0]
    c, h, w = fx.img.shape
    np.testing.assert_array_equal(eng.decode_window(fx.cs, (5, 7, w - 3, h - 11)), fx.img[:, 7:h - 11, 5:w - 3])
    with pytest.raises(RuntimeError):
        eng.decode_window(fx.cs, (0, 0, w + 1, h))


class _HostEngineCoder:
    """grok_amd.shard.EngineCoder behind host tensors: lets the gloo (CPU-tensor) collectives of
    two processes sharing this box's one GPU drive bench.py's runners with the real engine."""

    def __init__(self, shape, bits, params):
        import grok_amd as G
        from grok_amd import shard
        self.eng = G.Engine(0)
        self.ec = shard.EngineCoder(self.eng, shape, bits, params)

    def main_header(self):
        return self.ec.main_header()

    def encode_tiles(self, x, tb, te, row0, out):
        import torch
        od = torch.empty(out.numel(), dtype=torch.uint8, device="cuda")
        n, lens = self.ec.encode_tiles(x.cuda(), tb, te, row0, od)
        out[:n] = od[:n].cpu()
        return n, lens

    def decode_rows(self, sub, n, out, row0):
        import torch
        od = torch.empty(out.shape, dtype=out.dtype, device="cuda")
        self.ec.decode_rows(sub[:n].cuda(), n, od, row0)
        out.copy_(od.cpu())

    def decode_window(self, cs, n, win, out):
        import torch
        od = torch.empty(out.shape, dtype=out.dtype, device="cuda")
        self.ec.decode_window(cs[:n].cuda(), n, win, od)
        out.copy_(od.cpu())


def _bench_runner_worker(rank, world, port, q):
    import os
    import sys
    import torch
    import torch.distributed as dist
    sys.path.insert(0, ROOT)
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import bench
        import grok_amd as G
        from grok_amd.synth import synth_image
        size, tiles = 512, (128, 128)
        bench.CONFIGS["C4"] = dict(bench.CONFIGS["C4"], params=dict(bench.CONFIGS["C4"]["params"], tiles=tiles))
        cfg = bench.CONFIGS["C4"]
        coder = _HostEngineCoder((1, size, size), 16, G.default_params(**cfg["params"]))
        r = bench.ShardRunner("C4", size, rank, world, torch.device("cpu"), dist, coder=coder)
        r.check()
        ok4 = True
        if rank == 0:
            img = synth_image(size, size, 1, 16, cfg["seed"]).astype(np.int32)
            ok4 = r.cs[:r.n].numpy().tobytes() == O.encode(img, 16, cblk_sty=64, tiles=tiles, tlm=True, plt=True)
        # C5: windows of a tiled RGB8 .jp2 on rank 0, each rank given only its band's tile parts
        S = 384
        kw5 = dict(tiles=(128, 128), tlm=True, plt=True, jp2=True)
        img5 = synth_image(S, S, 3, 8, 30).astype(np.int32)
        file = n = None
        if rank == 0:
            cs = O.encode(img5, 8, **kw5)
            file, n = torch.frombuffer(bytearray(cs), dtype=torch.uint8), len(cs)
        wins = [(0, 0, 128, 128), (37, 50, 301, 350), (300, 300, 384, 384)]
        coder5 = _HostEngineCoder((3, S, S), 8, G.default_params(tiles=(128, 128), tlm=True, plt=True, jp2=True))
        r5 = bench.C5Runner(rank, world, torch.device("cpu"), dist, size=S, windows=wins, coder=coder5, file=file, n=n)
        r5.check()
        ok5 = True
        if rank == 0:
            ok5 = all(np.array_equal(o.numpy(), img5[:, y0:y1, x0:x1]) for o, (x0, y0, x1, y1) in zip(r5.outs, wins))
            q.put((bool(ok4), bool(ok5)))
        coder.eng.close()
        coder5.eng.close()
    finally:
        dist.destroy_process_group()


def test_bench_runners_two_processes_one_gpu():
    # bench.py's ShardRunner (C4) and C5Runner step() with the HIP engine in two rank processes
    import socket
    import torch.multiprocessing as mp
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_bench_runner_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res == (True, True)


def test_bench_runners_world1_device():
    # the same runners at world size 1 on device tensors (the collective-free path bench.py takes on one GPU)
    import torch
    import bench
    from grok_amd.synth import synth_image
    dev = torch.device("cuda", 0)
    r = bench.ShardRunner("C4", 2048, 0, 1, dev, None)
    r.check()
    r.close()
    r5 = bench.C5Runner(0, 1, dev, None, size=4096, windows=[(0, 0, 1024, 1024), (1234, 2345, 3001, 4000)])
    r5.check()
    r5.close()
