"""Benchmark: Mpixels/s encode+decode, JPEG 2000 tile pipeline on MI355X.

Workload (BASELINE.json configs[1], "C2"): 8192x8192 8-bit RGB, 5/3 reversible
lossless + RCT, 64x64 code-blocks, 6 resolutions, single tile, one quality
layer — Grok's default coding parameters.  Synthetic input from the survey's
seeded generator (grok_amd/synth.py, seed 10).

One step = encode (image resident in HBM -> codestream resident in HBM) +
decode (codestream in HBM -> image in HBM), with the host doing T2 packet
headers from per-block metadata.  value = pixels of all ranks / max-over-ranks
wall time.  Single-tile configs shard as replicas (one image per GPU, no
collective): scaling = "weak".

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--size", type=int, default=8192)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=1024, help="side of the CPU-baseline crop")
    return ap.parse_args()


def cpu_baseline(img, side):
    """Oracle (CPU restatement, bit-exact with Grok) on a bounded crop, 1 thread."""
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "oracle"))
    import oracle as O
    crop = np.ascontiguousarray(img[:, :side, :side]).astype(np.int32)
    t0 = time.perf_counter()
    cs = O.encode(crop, 8)
    t1 = time.perf_counter()
    dec, _ = O.decode(cs)
    t2 = time.perf_counter()
    assert (dec == crop).all()
    mpix = side * side / 1e6
    return {"value": mpix / (t2 - t0), "unit": "Mpixels/s", "cores": 1, "kind": "port",
            "sample": "%dx%d RGB8 crop of the C2 image, oracle enc %.2fs + dec %.2fs, 1 thread" % (
                side, side, t1 - t0, t2 - t1)}


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
    import grok_amd as G
    from grok_amd.synth import synth_image

    S = args.size
    img = synth_image(S, S, 3, 8, 10 + rank)          # one independent image per rank (replicas)
    x = torch.from_numpy(img.astype(np.int32)).to(f"cuda:{local}").contiguous()
    out_cs = torch.empty(3 * S * S * 4 + (1 << 24), dtype=torch.uint8, device=f"cuda:{local}")
    y = torch.empty_like(x)
    eng = G.Engine(local)
    params = G.default_params()

    def step():
        n = eng.encode(x, 8, params=params, out=out_cs)
        te = eng.timings()
        eng.decode(out_cs, length=n, out=y)
        td = eng.timings()
        return n, te, td

    # correctness gate before timing
    n, te, td = step()
    torch.cuda.synchronize()
    if not torch.equal(x, y):
        raise SystemExit("lossless round trip FAILED on rank %d" % rank)
    for _ in range(args.warmup):
        step()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    dwt_ms, dwt_bytes, t1e, t1d = 0.0, 0, 0.0, 0.0
    for _ in range(args.steps):
        n, te, td = step()
        dwt_ms += te.dwt_ms + td.dwt_ms
        dwt_bytes += te.dwt_bytes + td.dwt_bytes
        t1e += te.t1_ms
        t1d += td.t1_ms
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    el = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([el], device=f"cuda:{local}")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        el = float(t.item())
    ms = el * 1000.0 / args.steps
    mpix = S * S / 1e6
    value = mpix * world * args.steps / el
    if rank == 0:
        achieved = (dwt_bytes / 1e9) / (dwt_ms / 1e3) if dwt_ms > 0 else 0.0
        res = {
            "metric": "Mpixels/s encode+decode, 8K RGB 5/3 lossless + 9/7 lossy, 1/2/4/8 GPU",
            "value": round(value, 3), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "int32", "data": "synthetic (seeded survey generator, seed 10+rank)",
            "config": {"workload": "C2: %dx%d 8-bit RGB, 5/3 lossless + RCT, 64x64 code-blocks, 6 resolutions, "
                                   "single tile, 1 layer; encode+decode, image and codestream resident in HBM" % (S, S),
                       "parallelism": "replicas x%d" % world, "codestream_bytes": int(n)},
            "roofline": {"bound": "hbm", "kernel": "k_dwt53_fwd_level + k_dwt53_inv_level (all levels)",
                         "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None},
            "stages_ms": {"enc_mct": round(te.mct_ms, 3), "enc_dwt": round(te.dwt_ms, 3), "enc_t1": round(te.t1_ms, 3), "enc_t1_cm": round(te.t1_cm_ms, 3),
                          "enc_t2_host": round(te.t2_ms, 3), "enc_assemble": round(te.assemble_ms, 3),
                          "dec_t2_host": round(td.t2_ms, 3), "dec_t1": round(td.t1_ms, 3), "dec_dwt": round(td.dwt_ms, 3),
                          "dec_mct": round(td.mct_ms, 3)},
            "t1": {"blocks": te.t1_blocks, "enc_blocks_per_s": round(te.t1_blocks / (t1e / args.steps / 1e3), 1),
                   "dec_blocks_per_s": round(td.t1_blocks / (t1d / args.steps / 1e3), 1)},
        }
        if not args.no_cpu_baseline:
            res["cpu_baseline"] = cpu_baseline(img, args.cpu_sample)
        print(json.dumps(res), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
