"""Grid kernel against the BVH kernel on the reference's shipped Grid-default scenes (SURVEY.md §8
row f4: "Grid kernel perf parity with BVH — default accel of 5 shipped scenes").

For each of the five scenes whose P3F says `accel grid` (assignment1, balls_box, balls_high,
blueDiamond, dragon) the same scene text is rendered with `accel grid` and with `accel bvh`, in the
scene's own frame mode (Whitted, spp 0) at its own resolution and as a 16-spp AA frame, and
timed by the path kernel's HIP events over `--frames` frames (median).  Rays = closest + shadow
traversals of a stats frame; Mrays/s = rays / kernel ms.  The two accelerators do different work
for the same rays (a cell of the Grid can hold hundreds of triangles the BVH never tests), so the
line also carries each kernel's work counts and its rate of algorithmic record bytes (64 B per
inner-node visit + 48 B per object test), the kernel-efficiency comparison.  One JSON line per
(scene, mode).

  python tools/grid_vs_bvh.py [--frames 30] > gpurun_out/grid_vs_bvh.jsonl
"""
import argparse
import json
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import distributionraytracer_amd as drt  # noqa: E402
import shipped  # noqa: E402

SCENES = ("assignment1", "balls_box", "balls_high", "blueDiamond", "dragon")


def measure(r, tmp, name, accel, spp, frames):
    over = {"accel": accel} if spp is None else {"accel": accel, "spp": spp}
    d = Path(tmp) / f"{accel}_{spp}"
    d.mkdir(exist_ok=True)
    s = drt.Scene.load_p3f(shipped.write(d, name, **over), skybox_faces=shipped.skybox_faces(name))
    s.build()
    r.upload(s)
    img = r.render(seed=7, stats=True)
    st = r.stats()
    rays = st["closest_rays"] + st["shadow_rays"]
    for _ in range(3):
        r.render(seed=7)
    for _ in range(frames):
        r.render(seed=7)
    path_ms, _ = r.frame_times(frames)
    ms = float(np.median(path_ms[-frames:]))
    inner = st["closest_inner"] + st["shadow_inner"]  # BVH inner-node visits (0 on the Grid)
    cells = st["closest_leaf"] + st["shadow_leaf"]    # BVH leaf visits / Grid cells examined
    prims = st["closest_prims"] + st["shadow_prims"]  # Object::hit calls
    # algorithmic record bytes: 64 B per inner-node visit, 48 B per object test
    nbytes = 64 * inner + 48 * prims
    return dict(rays=int(rays), kernel_ms=round(ms, 4), mrays_s=round(rays / ms / 1e3, 1),
                inner=int(inner), leaf_or_cells=int(cells), prims=int(prims),
                gtests_s=round((inner + prims) / ms / 1e6, 2), record_GB_s=round(nbytes / ms / 1e6, 1)), img


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=30)
    ap.add_argument("--scenes", default=",".join(SCENES))
    ap.add_argument("--modes", default="whitted,aa16")
    args = ap.parse_args()
    r = drt.Renderer(0)
    with tempfile.TemporaryDirectory() as tmp:
        for name in args.scenes.split(","):
            for mode, spp in (("whitted", None), ("aa16", 16)):
                if mode not in args.modes.split(","):
                    continue
                g, gi = measure(r, tmp, name, "grid", spp, args.frames)
                b, bi = measure(r, tmp, name, "bvh", spp, args.frames)
                # the two accelerators' frames agree (tie-breaking between equal-t objects may differ)
                diff = float(np.mean(np.any(np.abs(gi - bi) > 1e-4, axis=2)))
                print(json.dumps({"scene": name, "mode": mode, "res": list(s for s in gi.shape[1::-1]),
                                  "grid": g, "bvh": b, "grid_over_bvh": round(g["mrays_s"] / b["mrays_s"], 3),
                                  # frame-time ratio (rays differ between one- and two-pass Whitted frames,
                                  # whose light samples share one closest-hit chain per pixel)
                                  "grid_speed_over_bvh": round(b["kernel_ms"] / g["kernel_ms"], 3),
                                  "grid_over_bvh_record_rate": round(g["record_GB_s"] / b["record_GB_s"], 3),
                                  "pixels_differing_frac": round(diff, 5)}), flush=True)
    r.close()


if __name__ == "__main__":
    main()
