"""Benchmark: Mpixels/s encode+decode, JPEG 2000 tile pipeline on MI355X.

Headline workload (BASELINE.json configs[1], "C2"): 8192x8192 8-bit RGB, 5/3
reversible lossless + RCT, 64x64 code-blocks, 6 resolutions, single tile, one
quality layer — Grok's default coding parameters.  Synthetic input from the
survey's seeded generator (grok_amd/synth.py, seed 10 + rank).

One step = encode (image resident in HBM -> codestream resident in HBM) +
decode (codestream in HBM -> image in HBM); host T2 (packet headers, rate
allocation) runs inside the step.  value = pixels of all ranks / max-over-ranks
wall time.  Single-tile configs shard as replicas (one image per GPU, no
collective on the data path): scaling = "weak".

The same JSON line carries auxiliary measurements of configs[2] ("C3":
8192x8192 12-bit RGB, 9/7 + ICT, 3 quality layers -r 40,20,10) and configs[3]
("C4": 16384x16384 16-bit mono, HTJ2K, 1024x1024 tiles, TLM + PLT).  With
N > 1 ranks C4 is tile-sharded (strong scaling): each rank codes its tile rows
from its own slab, rank 0 gathers the tile parts over RCCL and assembles the
codestream; each rank then decodes its own tile parts.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--config C2|C3] [--no-aux]
"""
import argparse
import glob
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8 TB/s peak

CONFIGS = {
    "C2": dict(size=8192, comps=3, bits=8, seed=10, params=dict(),
               desc="8192x8192 8-bit RGB, 5/3 lossless + RCT, 64x64 code-blocks, 6 resolutions, single tile, 1 layer"),
    "C3": dict(size=8192, comps=3, bits=12, seed=11, params=dict(irreversible=True, layer_rate=[40.0, 20.0, 10.0]),
               desc="8192x8192 12-bit RGB, 9/7 + ICT, 64x64 code-blocks, 6 resolutions, single tile, "
                    "3 layers -r 40,20,10 (PCRD)"),
    "C4": dict(size=16384, comps=1, bits=16, seed=20,
               params=dict(cblk_sty=0x40, tiles=(1024, 1024), tlm=True, plt=True),
               desc="16384x16384 16-bit mono, HTJ2K, 5/3 lossless, 1024x1024 tiles, TLM + PLT (-M 64 -t 1024,1024 -X -L)"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=0, help="override the config's image side")
    ap.add_argument("--config", default="C2", choices=sorted(CONFIGS))
    ap.add_argument("--no-aux", action="store_true", help="skip the auxiliary C3 measurement")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=2048, help="side of the CPU-baseline crop")
    return ap.parse_args()


def cpu_baseline(img, bits, side, params):
    """The oracle (CPU restatement, byte-exact with Grok), one thread, on a bounded crop."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle as O
    crop = np.ascontiguousarray(img[:, :side, :side]).astype(np.int32)
    kw = {}
    if params.get("irreversible"):
        kw = dict(irreversible=True, layer_rate=params.get("layer_rate"))
    t0 = time.perf_counter()
    cs = O.encode(crop, bits, **kw)
    t1 = time.perf_counter()
    dec, _ = O.decode(cs)
    t2 = time.perf_counter()
    if not kw:
        assert (dec == crop).all()
    mpix = side * side / 1e6
    return {"value": round(mpix / (t2 - t0), 4), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": "%dx%d crop of the same image, oracle/j2k_oracle.cpp encode %.2fs + decode %.2fs, 1 thread" % (
                side, side, t1 - t0, t2 - t1)}


def pmc_traffic(kernels):
    """HBM bytes per launch of `kernels` from the newest committed PMC summary
    (profiles/*_pmc.json, written by tools/pmc_summary.py from rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes of this benchmark; FETCH_SIZE doubled per
    MI355X_MICROARCH.md's gfx950 note).  None if no summary exists."""
    files = sorted(glob.glob(os.path.join(ROOT, "profiles", "*_pmc.json")))
    if not files:
        return None
    d = json.load(open(files[-1]))
    tot = 0.0
    for k in kernels:
        if k not in d:
            return None
        tot += d[k]["hbm_bytes_per_launch"]
    return tot


class Runner:
    def __init__(self, name, size, rank, device):
        import torch
        import grok_amd as G
        from grok_amd.synth import synth_image
        cfg = CONFIGS[name]
        size = size or cfg["size"]
        self.name, self.cfg, self.size = name, cfg, size
        self.img = synth_image(size, size, cfg["comps"], cfg["bits"], cfg["seed"] + rank)
        self.x = torch.from_numpy(self.img.astype(np.int32)).to(device).contiguous()
        self.out = torch.empty(self.x.numel() * 4 + (1 << 24), dtype=torch.uint8, device=device)
        self.y = torch.empty_like(self.x)
        self.eng = G.Engine(device.index or 0)
        self.params = G.default_params(**cfg["params"])
        self.n = 0

    def step(self):
        self.n = self.eng.encode(self.x, self.cfg["bits"], params=self.params, out=self.out)
        te = self.eng.timings()
        self.eng.decode(self.out, length=self.n, out=self.y)
        td = self.eng.timings()
        return te, td

    def check(self):
        import torch
        self.step()
        torch.cuda.synchronize()
        if not self.cfg["params"].get("irreversible"):
            if not torch.equal(self.x, self.y):
                raise SystemExit("lossless round trip FAILED (%s)" % self.name)
        else:
            d = (self.y - self.x).double()
            mse = float((d * d).mean())
            psnr = 10 * np.log10(((1 << self.cfg["bits"]) - 1) ** 2 / mse)
            if psnr < 30.0:
                raise SystemExit("9/7 round trip PSNR %.2f dB too low (%s)" % (psnr, self.name))
            return psnr
        return None


class BatchRunner:
    """`nimg` images in flight on one GPU: each has its own engine (own HIP stream and
    buffers) and is driven from its own host thread, so one image's host T2 and
    chain-bound T1 kernels overlap with the other's (ctypes releases the GIL).  One
    step = every image encoded and decoded once.  Image i uses seed cfg.seed + rank
    + 1000 * i (same generator, same statistics)."""

    def __init__(self, name, nimg, rank, device):
        from concurrent.futures import ThreadPoolExecutor
        self.rs = [Runner(name, 0, rank + 1000 * i, device) for i in range(nimg)]
        self.size, self.cfg, self.name = self.rs[0].size, self.rs[0].cfg, name
        self.n = self.rs[0].n
        self.pool = ThreadPoolExecutor(nimg)

    def step(self):
        res = [f.result() for f in [self.pool.submit(r.step) for r in self.rs]]
        self.n = self.rs[0].n
        return res[0]

    def check(self):
        for r in self.rs:
            r.check()
        self.n = self.rs[0].n

    def close(self):
        self.pool.shutdown()
        for r in self.rs:
            r.eng.close()


class ShardRunner:
    """C4 on N ranks: tile rows split across ranks (grok_amd/shard.py).  One step =
    every rank encodes its tiles from its slab (HBM -> tile parts in HBM), rank 0
    gathers the tile parts (RCCL) and assembles the codestream in HBM, every rank
    decodes its own tile parts back into its slab."""

    def __init__(self, name, size, rank, world, device, dist):
        import torch
        import grok_amd as G
        from grok_amd import shard
        from grok_amd.synth import synth_slab
        cfg = CONFIGS[name]
        size = size or cfg["size"]
        self.name, self.cfg, self.size, self.rank, self.world, self.dist = name, cfg, size, rank, world, dist
        self.device = device
        tw, th = cfg["params"]["tiles"]
        self.ntx, self.nty = shard.tile_grid(size, size, th, tw)
        self.tb, self.te, j0, j1 = shard.rank_tiles(self.ntx, self.nty, rank, world)
        if self.te <= self.tb:
            raise SystemExit("C4 sharding needs at least one tile row per rank")
        self.y0, self.y1 = j0 * th, min(size, j1 * th)
        slab = synth_slab(self.y0, self.y1, size, size, cfg["comps"], cfg["bits"], cfg["seed"])
        self.x = torch.from_numpy(slab.astype(np.int32)).to(device).contiguous()
        self.y = torch.empty_like(self.x)
        self.eng = G.Engine(device.index or 0)
        self.params = G.default_params(**cfg["params"])
        hdr, self.tlm, _ = self.eng.main_header((cfg["comps"], size, size), cfg["bits"], params=self.params)
        self.hdr = torch.frombuffer(bytearray(hdr), dtype=torch.uint8).to(device)
        self.eoc = torch.tensor([0xFF, 0xD9], dtype=torch.uint8, device=device)
        self.parts = torch.empty(self.x.numel() * 4 + (1 << 22), dtype=torch.uint8, device=device)
        self.n = 0
        self.cs = None

    def step(self):
        import torch
        n, lens = self.eng.encode_tiles(self.x, self.cfg["bits"], self.tb, self.te, image_hw=(self.size, self.size),
                                        row0=self.y0, params=self.params, out=self.parts)
        te = self.eng.timings()
        # gather tile parts to rank 0 (lengths, then padded payload) over RCCL
        ln = torch.tensor([n], dtype=torch.int64, device=self.device)
        lns = [torch.zeros_like(ln) for _ in range(self.world)]
        self.dist.all_gather(lns, ln)
        mx = int(max(int(v.item()) for v in lns))
        payload = self.parts[:mx]
        if self.rank == 0:
            bufs = [torch.empty(mx, dtype=torch.uint8, device=self.device) for _ in range(self.world)]
            self.dist.gather(payload, bufs, dst=0)
            self.cs = torch.cat([self.hdr] + [b[:int(k.item())] for b, k in zip(bufs, lns)] + [self.eoc])
            self.n = int(self.cs.numel())
        else:
            self.dist.gather(payload, None, dst=0)
        # each rank decodes its own tile parts (main header + parts + EOC) into its slab
        sub = torch.cat([self.hdr, self.parts[:n], self.eoc])
        self.eng.decode(sub, length=int(sub.numel()), out=self.y, row0=self.y0)
        td = self.eng.timings()
        return te, td

    def check(self):
        import torch
        self.step()
        torch.cuda.synchronize()
        if not torch.equal(self.x, self.y):
            raise SystemExit("sharded lossless round trip FAILED (%s)" % self.name)
        return None


def timed(r, steps, warmup, world, dist, device):
    import torch
    for _ in range(warmup):
        r.step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    acc = {}
    for _ in range(steps):
        te, td = r.step()
        for pre, t in (("enc", te), ("dec", td)):
            for f, _ in t._fields_:
                acc[pre + "_" + f] = acc.get(pre + "_" + f, 0.0) + float(getattr(t, f))
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    return el, {k: v / steps for k, v in acc.items()}


def main():
    args = parse()
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl" if torch.cuda.is_available() else "gloo")
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)

    r = Runner(args.config, args.size, rank, device)
    S = r.size
    r.check()
    el, m = timed(r, args.steps, args.warmup, world, dist, device)
    ms = el * 1000.0 / args.steps
    samples = S * S * r.cfg["comps"]
    value = S * S / 1e6 * world * args.steps / el

    aux = None
    if not args.no_aux and args.config == "C2":
        aux = {}
        r.eng.close()
        del r.x, r.y, r.out
        torch.cuda.empty_cache()
        r3 = Runner("C3", args.size, rank, device)
        psnr = r3.check()
        el3, m3 = timed(r3, 2, 1, world, dist, device)
        S3 = r3.size
        aux["C3"] = {"config": "C3: " + CONFIGS["C3"]["desc"], "value": round(S3 * S3 / 1e6 * world * 2 / el3, 3),
                     "unit": "Mpixels/s", "ms_per_step": round(el3 * 500.0, 3), "psnr_db": round(psnr, 3),
                     "codestream_bytes": int(r3.n), "parallelism": "replicas x%d" % world,
                     "stages_ms": {k: round(v, 3) for k, v in m3.items() if k.endswith("_ms") and v > 0}}
        r3.eng.close()
        del r3
        torch.cuda.empty_cache()
        # C2 with two images in flight per GPU (throughput of overlapped independent jobs)
        rb = BatchRunner("C2", 2, rank, device)
        rb.check()
        elb, mb = timed(rb, 3, 1, world, dist, device)
        Sb = rb.size
        aux["C2_batch2"] = {"config": "C2 with 2 images in flight per GPU (2 engines / HIP streams, one host thread "
                                      "each); one step = 2 images encoded + decoded",
                            "value": round(2 * Sb * Sb / 1e6 * world * 3 / elb, 3), "unit": "Mpixels/s",
                            "ms_per_step": round(elb * 1000.0 / 3, 3), "images_per_step": 2,
                            "parallelism": "replicas x%d" % world}
        rb.close()
        del rb
        torch.cuda.empty_cache()
        r4 = ShardRunner("C4", 0, rank, world, device, dist) if world > 1 else Runner("C4", 0, rank, device)
        r4.check()
        el4, m4 = timed(r4, 3, 1, world, dist, device)
        S4 = r4.size
        aux["C4"] = {"config": "C4: " + CONFIGS["C4"]["desc"], "value": round(S4 * S4 / 1e6 * 3 / el4, 3),
                     "unit": "Mpixels/s", "ms_per_step": round(el4 * 1000.0 / 3, 3),
                     "codestream_bytes": int(r4.n),
                     "parallelism": ("tile rows sharded over %d ranks, RCCL gather of tile parts to rank 0" % world)
                     if world > 1 else "1 GPU, all 256 tiles batched",
                     "scaling": "strong",
                     "stages_ms": {k: round(v, 3) for k, v in m4.items() if k.endswith("_ms") and v > 0},
                     "t1_blocks": int(m4.get("enc_t1_blocks", 0))}
        r4.eng.close()

    if rank == 0:
        # dominant kernel: the T1 stage with the largest average duration, measured with HIP
        # events on the engine stream (encode: k_t1_cm + k_t1_mq, decode: k_t1_dec2 + k_t1_recon)
        stages = {
            "T1 decode (k_t1_dec2 + k_t1_recon)": (m["dec_t1_ms"], m["dec_t1_bytes"] + 4.0 * samples,
                                                   ["void k_t1_dec2<false>", "k_t1_recon"]),
            "T1 encode (k_t1_cm + k_t1_mq)": (m["enc_t1_ms"], 4.0 * samples + m["enc_t1_bytes"],
                                              ["void k_t1_cm<false>", "k_t1_mq"]),
            "DWT 5/3 fwd+inv (all levels)": (m["enc_dwt_ms"] + m["dec_dwt_ms"], m["enc_dwt_bytes"] + m["dec_dwt_bytes"],
                                             ["k_dwt53_fwd_level", "k_dwt53_inv_level"]),
        }
        dom = max(stages, key=lambda k: stages[k][0])
        t_ms, nbytes, kern = stages[dom]
        achieved = nbytes / 1e9 / (t_ms / 1e3)
        traffic = pmc_traffic(kern)
        dwt_gbs = (m["enc_dwt_bytes"] + m["dec_dwt_bytes"]) / 1e9 / ((m["enc_dwt_ms"] + m["dec_dwt_ms"]) / 1e3)
        res = {
            "metric": "Mpixels/s encode+decode, 8K RGB 5/3 lossless + 9/7 lossy, 1/2/4/8 GPU",
            "value": round(value, 3), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32",
            "data": "synthetic (seeded survey generator grok_amd/synth.py, seed %d+rank)" % r.cfg["seed"],
            "config": {"workload": "%s: %s; encode+decode, image and codestream resident in HBM" % (
                args.config, r.cfg["desc"]), "parallelism": "replicas x%d (one image per GPU)" % world,
                "codestream_bytes": int(r.n)},
            "roofline": {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 5),
                         "traffic": None if traffic is None else round(traffic),
                         "bytes_per_launch": round(nbytes), "avg_ms": round(t_ms, 3),
                         "note": "T1 is a serial MQ chain per code-block; bytes = compressed bytes + 4 B/sample"},
            "dwt_roofline": {"achieved": round(dwt_gbs, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                             "frac": round(dwt_gbs / HBM_PEAK_GBS, 4), "bytes_per_sample": 10.656},
            "stages_ms": {k: round(v, 3) for k, v in m.items() if k.endswith("_ms") and v > 0},
            "t1": {"blocks": int(m["enc_t1_blocks"]),
                   "enc_blocks_per_s": round(m["enc_t1_blocks"] / (m["enc_t1_ms"] / 1e3)),
                   "dec_blocks_per_s": round(m["dec_t1_blocks"] / (m["dec_t1_ms"] / 1e3))},
        }
        if aux:
            res["aux"] = aux
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(r.img, r.cfg["bits"], min(args.cpu_sample, S), r.cfg["params"])
        print(json.dumps(res), flush=True)
    if aux is None:
        r.eng.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
