"""Whitted frames (spp 0) of the reference's shipped scenes in one pass against two passes (round 5:
MODE_CHAIN traces each pixel's closest-hit chain, MODE_AREPLAY shades every (pixel, light sample)
with its shadow queries on the shadow tree / the Grid).  Per scene and resolution: the plan each way,
the median path-kernel time of --frames frames (HIP events), and whether the frames are bit-identical.
Scenes with a refracting material keep one pass either way (drt_capi.hip plan).

  python tools/whitted_two_pass.py [--frames 20] [--res 1024] > gpurun_out/whitted_two_pass.jsonl
"""
import argparse
import json
import os
import sys
import tempfile
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
sys.path.insert(0, str(ROOT / "tests"))

import distributionraytracer_amd as drt  # noqa: E402
import shipped  # noqa: E402

SCENES = ("dragon_assignment1", "dragon", "assignment1", "balls_high", "balls_box", "blueDiamond")


def run(r, frames):
    r.render(seed=7)
    for _ in range(frames):
        r.render(seed=7)
    path_ms, _ = r.frame_times(frames)
    return float(np.median(path_ms))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--frames", type=int, default=20)
    ap.add_argument("--res", default="native,1024")
    ap.add_argument("--scenes", default=",".join(SCENES))
    args = ap.parse_args()
    r = drt.Renderer(0)
    with tempfile.TemporaryDirectory() as tmp:
        for name in args.scenes.split(","):
            for res in args.res.split(","):
                over = {} if res == "native" else {"res": (int(res), int(res))}
                d = Path(tmp) / f"{name}_{res}"
                d.mkdir()
                s = drt.Scene.load_p3f(shipped.write(d, name, **over), skybox_faces=shipped.skybox_faces(name))
                s.build()
                r.upload(s)
                row = {"scene": name, "res": list(r.render(seed=7).shape[1::-1]), "accel": s.info().accel}
                out = {}
                for label, env in (("one_pass", {"DRT_WHITTED_TWO_PASS": "0"}), ("default", {}),
                                   ("two_pass", {"DRT_AA_TWO_PASS": "2"})):
                    old = {k: os.environ.get(k) for k in ("DRT_WHITTED_TWO_PASS", "DRT_AA_TWO_PASS")}
                    os.environ.update(env)
                    try:
                        plan = r.plan(r.frame_params(seed=7))["passes"]
                        img = r.render(seed=7)
                        ms = run(r, args.frames)
                    finally:
                        for k, v in old.items():
                            if v is None:
                                os.environ.pop(k, None)
                            else:
                                os.environ[k] = v
                    out[label] = img
                    row[label] = {"passes": plan, "path_ms": round(ms, 4)}
                row["identical"] = bool(np.array_equal(out["one_pass"].view(np.uint32), out["two_pass"].view(np.uint32)) and
                                        np.array_equal(out["one_pass"].view(np.uint32), out["default"].view(np.uint32)))
                row["two_over_one"] = round(row["two_pass"]["path_ms"] / row["one_pass"]["path_ms"], 3)
                print(json.dumps(row), flush=True)
    r.close()


if __name__ == "__main__":
    main()
