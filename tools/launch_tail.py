#!/usr/bin/env python3
"""The tail of a persistent launch, from per-wave start / end stamps (drt_frame_wave_times, round 6).

Renders one stats frame of a BASELINE workload and reports, for its pass-1 persistent launch (C4: the
in-order MODE_SKEL closest-chain pass, main.cpp:650-665; the headline: the AA MODE_CHAIN pass) and, where
there is one, its pass-2 persistent launch (the Grid's shadow-query stream):
  - the launch span and the distribution of wave end times (percentiles of the span);
  - `busy_frac`: the wave-time the waves were alive over (waves x span) — 1 - busy_frac is the share of
    the launch's wave slots idle because their wave had run out of work (the tail);
  - `tail_ms`: the time from the 50 % / 90 % wave end to the last one.
Workloads as bench.py names them (its flags).  GPU only.

    python tools/launch_tail.py [bench.py workload flags, e.g. --res 1024 --aperture 8 --focal 1 --roughness 0.1 --max-depth 8]
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402


def summarize(w):
    if len(w) == 0:
        return None
    t0 = w[:, 0].min()
    ends = np.sort(w[:, 1] - t0)
    span = ends[-1]
    q = {p: round(float(np.percentile(ends, p)) / 1e3, 3) for p in (10, 50, 90, 99, 100)}
    busy = float((w[:, 1] - w[:, 0]).sum() / (len(w) * span)) if span > 0 else 1.0
    return {"waves": int(len(w)), "span_ms": round(float(span) / 1e3, 3), "wave_end_ms_percentiles": q,
            "busy_frac": round(busy, 4), "tail_ms_after_p50": round(float(span - np.percentile(ends, 50)) / 1e3, 3),
            "tail_ms_after_p90": round(float(span - np.percentile(ends, 90)) / 1e3, 3)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--spp", type=int, default=64)
    ap.add_argument("--aperture", type=float, default=0.0)
    ap.add_argument("--focal", type=float, default=1.0)
    ap.add_argument("--roughness", type=float, default=0.0)
    ap.add_argument("--max-depth", type=int, default=4)
    ap.add_argument("--light-spp", type=int, default=1)
    ap.add_argument("--accel", default="bvh")
    ap.add_argument("--frames", type=int, default=2, help="stats frames (the last one is reported)")
    a = ap.parse_args()

    import torch  # noqa: F401  (one HIP runtime for the library and torch)

    import distributionraytracer_amd as drt

    class Args:  # bench.make_scene's view of the command line
        scene = "synthetic"
        tris, res, spp, seed, ks = a.tris, a.res, a.spp, 1, 0.5
    ext = {"aperture": a.aperture, "focal": a.focal, "roughness": a.roughness, "max_depth": a.max_depth,
           "light_spp": a.light_spp, "accel": a.accel, "ks": 0.5}
    s = bench.make_scene(drt, Args, bench.synthetic_triangles(a.tris, 1), ext)
    s.build()
    r = drt.Renderer(0)
    try:
        r.upload(s)
        kw = {"max_depth": a.max_depth, "roughness": a.roughness, "light_spp": a.light_spp}
        plan = r.plan(r.frame_params(seed=1, **kw))
        for _ in range(a.frames):
            r.render(seed=1, stats=True, **kw)
        p1, p2 = r.frame_pass_times(1)
        out = {"workload": vars(a), "plan": plan, "pass_ms": [round(float(p1[0]), 3), round(float(p2[0]), 3)],
               "pass1": summarize(r.wave_times(0))}
        if plan["passes"] == 2:
            out["pass2"] = summarize(r.wave_times(1))
        print(json.dumps(out))
    finally:
        r.close()


if __name__ == "__main__":
    main()
