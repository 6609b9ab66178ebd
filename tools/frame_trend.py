#!/usr/bin/env python3
"""Per-frame device time over a long run of the bench workload (clock ramp / thermal trend):
frames rendered back to back with two in flight, the interval between consecutive frame ends
(HIP events) printed per frame.  usage: python tools/frame_trend.py [frames]"""
import sys
import time
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import bench  # noqa: E402


def main():
    import types

    import torch

    import distributionraytracer_amd as drt

    n = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    args = types.SimpleNamespace(scene="synthetic", res=512, spp=64)
    s = bench.make_scene(drt, args, bench.synthetic_triangles(1_000_000, 1),
                         {"aperture": 0.0, "focal": 1.0, "accel": "bvh", "ks": 0.5})
    s.build()
    r = drt.Renderer(0)
    r.upload(s)
    streams = [torch.cuda.current_stream(), torch.cuda.Stream()]
    outs = [torch.empty((512, 512, 3), dtype=torch.float32, device="cuda") for _ in range(2)]
    ps = [r.frame_params(seed=1, slot=j) for j in range(2)]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        j = i % 2
        r.render_device(ps[j], outs[j].data_ptr(), streams[j].cuda_stream)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    a, b, e = r.frame_spans(n)
    iv = np.diff(np.concatenate([[0.0], np.sort(e)]))
    print(f"{n} frames in {wall * 1e3:.1f} ms wall; per-frame interval ms:")
    print(" ".join(f"{x:.1f}" for x in iv))
    print(f"first 5 mean {iv[:5].mean():.2f}, last 10 mean {iv[-10:].mean():.2f}")


if __name__ == "__main__":
    main()
