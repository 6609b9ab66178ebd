"""Raw stats of one headline-scene frame (any accelerator) as JSON: python tools/grid_diag.py [--accel grid]
With DRT_LIBRARY=.../libdrt_gdiag.so (make variant NAME=gdiag EXTRA_HIPFLAGS=-DDRT_GRID_DIAG) the Grid
stepper also reports lane cell visits (cycles_leaf), pair-loop wave iterations (wave_leaf_iters), walk
lane steps (stack_pushes) and walk wave iterations (stack_spills)."""
import argparse
import json
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1]))
import torch  # noqa: F401,E402

import bench  # noqa: E402
import distributionraytracer_amd as drt  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--accel", default="grid")
ap.add_argument("--tris", type=int, default=1_000_000)
ap.add_argument("--res", type=int, default=512)
ap.add_argument("--spp", type=int, default=64)
a = ap.parse_args()
s = drt.Scene()
bench.populate(s, bench.synthetic_triangles(a.tris), a.res, a.spp, accel=a.accel)
s.build()
r = drt.Renderer(0)
r.upload(s)
r.render(seed=1, stats=True)
st = r.stats()
print(json.dumps(st))
