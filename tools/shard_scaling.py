#!/usr/bin/env python3
"""Per-rank frame time of an N-way tile-sharded frame, measured on ONE GPU.

bench.py --gpus N gives each rank the tiles t = rank + k*N of the frame.  Rendering one such
shard alone on one MI355X (drt_render_device with n_shards = N) is what each GPU of an N-GPU
run computes, minus the all-gather: T(1) / (N * T(N)) bounds the strong-scaling efficiency the
multi-GPU bench can reach (tail of the persistent kernel, per-frame launch and reduce costs).

    python tools/shard_scaling.py [--tris 1000000] [--res 512] [--spp 64] [--steps 5]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--shards", default="1,2,4,8")
    ap.add_argument("--pipe", type=int, default=1, help="frames in flight (bench.py --frames-in-flight)")
    ap.add_argument("--all-shards", action="store_true", help="time every shard, not just the first and last")
    ap.add_argument("--tile", type=int, default=16, help="tile edge in pixels (drt_frame_params.tile)")
    args = ap.parse_args()

    import torch

    import distributionraytracer_amd as drt

    scene = drt.Scene()
    bench.populate(scene, bench.synthetic_triangles(args.tris, 1), args.res, args.spp)
    scene.build()
    r = drt.Renderer(0)
    r.upload(scene)
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(args.pipe - 1)]
    out = {"tris": args.tris, "res": args.res, "spp": args.spp, "pipe": args.pipe, "tile": args.tile, "per_shard": {}}
    t1 = None
    for n in (int(x) for x in args.shards.split(",")):
        worst = 0.0
        rec = {}
        for shard in (range(n) if args.all_shards else sorted({0, n - 1})):
            ps = [r.frame_params(seed=1, shard=shard, n_shards=n, slot=j, tile=args.tile) for j in range(args.pipe)]
            _, floats = r.shard_layout(ps[0])
            bufs = [torch.empty(floats, dtype=torch.float32, device="cuda") for _ in range(args.pipe)]
            for i in range(2):
                j = i % args.pipe
                r.render_device(ps[j], bufs[j].data_ptr(), streams[j].cuda_stream)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for i in range(args.steps):
                j = i % args.pipe
                r.render_device(ps[j], bufs[j].data_ptr(), streams[j].cuda_stream)
            torch.cuda.synchronize()
            ms = (time.perf_counter() - t0) / args.steps * 1e3
            path_ms, _ = r.frame_times(args.steps)
            rec[f"shard{shard}"] = {"frame_ms": round(ms, 3), "kernel_ms": round(float(path_ms.mean()), 3)}
            worst = max(worst, ms)
        if n == 1:
            t1 = worst
        rec["efficiency_bound"] = round(t1 / (n * worst), 3) if t1 else None
        out["per_shard"][n] = rec
        print(n, json.dumps(rec), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
