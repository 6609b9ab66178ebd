#!/usr/bin/env python3
"""Traversal-only throughput of the streaming BVH kernel (drt_trace_closest / drt_trace_shadow).

Builds bench.py's scene (N random triangles + floor, BVH), makes a ray population like the
bench frame's — jittered primary rays, shadow rays from their hits to a quad-light point and
the point light, mirror-reflection rays — and times each set on the streaming kernel at 6, 7
and 8 waves per SIMD (HIP events around the kernel).  Node steps = inner visits + leaf visits.

    python tools/trace_bench.py [--tris 1000000] [--res 512] [--spp 4]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

import numpy as np

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))

import bench  # noqa: E402  (scene helpers)


def primary_rays(cam, res, spp, rng):
    eye = np.array(cam.eye, np.float32)
    u, v, n = (np.array(x, np.float32) for x in (cam.u, cam.v, cam.n))
    y, x = np.mgrid[0:res, 0:res].astype(np.float32)
    x = np.repeat(x.reshape(-1), spp) + rng.random(res * res * spp, dtype=np.float32)
    y = np.repeat(y.reshape(-1), spp) + rng.random(res * res * spp, dtype=np.float32)
    d = (u[None] * (cam.w * (x / res - 0.5))[:, None] + v[None] * (cam.h * (y / res - 0.5))[:, None]
         - n[None] * cam.plane_dist)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.broadcast_to(eye, d.shape)
    return np.concatenate([o, d], 1).astype(np.float32)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tris", type=int, default=1_000_000)
    ap.add_argument("--res", type=int, default=512)
    ap.add_argument("--spp", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--waves", default="6,7,8")
    ap.add_argument("--reference-order", action="store_true",
                    help="shadow queries on the reference's binary tree (DRT_FRAME_REFERENCE_ORDER)")
    args = ap.parse_args()

    import torch  # noqa: F401  (one HIP runtime: torch's)
    import distributionraytracer_amd as drt

    scene = drt.Scene()
    bench.populate(scene, bench.synthetic_triangles(args.tris, 1), args.res, 1)
    scene.build()
    r = drt.Renderer(0)
    r.upload(scene)
    rng = np.random.default_rng(5)
    prim = primary_rays(scene.camera_frame(), args.res, args.spp, rng)
    t, nrm, obj = r.trace_closest(prim)
    hit = obj >= 0
    o, d = prim[hit, :3], prim[hit, 3:]
    P = o + d * t[hit, None]
    N = nrm[hit] / np.linalg.norm(nrm[hit], axis=1, keepdims=True)
    N = np.where((np.sum(d * N, 1) < 0)[:, None], N, -N)
    so = P + N * np.float32(1e-4)
    lq = np.array([4, 3, 2], np.float32) + rng.random((len(P), 1), dtype=np.float32) * np.array([0, -1, 0], np.float32) \
        + rng.random((len(P), 1), dtype=np.float32) * np.array([-1, 0, 0], np.float32)
    sets = {
        "primary": (prim, False),
        "shadow_quad": (np.concatenate([so, lq - so], 1).astype(np.float32), True),
        "shadow_point": (np.concatenate([so, np.array([-3, 1, 5], np.float32) - so], 1).astype(np.float32), True),
        "reflect": (np.concatenate([so, d - 2 * np.sum(d * N, 1, keepdims=True) * N], 1).astype(np.float32), False),
    }
    out = {"tris": args.tris, "sets": {}}
    for name, (rays, shadow) in sets.items():
        fn = r.trace_shadow if shadow else r.trace_closest
        r.set_trace_stats(True, reference_order=args.reference_order)
        fn(rays)
        st = r.trace_stats()
        r.set_trace_stats(False, reference_order=args.reference_order)
        kind = "shadow" if shadow else "closest"
        # batched shadow queries walk the 4-ary shadow tree unless --reference-order
        inner = st[f"{kind}_inner"] + (st["wide_inner"] if shadow else 0)
        leaf = st[f"{kind}_leaf"] + (st["wide_leaf"] if shadow else 0)
        prims = st[f"{kind}_prims"] + (st["wide_prims"] if shadow else 0)
        steps = inner + leaf + (st["wide_verify"] if shadow else 0)
        rec = {"rays": len(rays), "inner_per_ray": inner / len(rays), "leaf_per_ray": leaf / len(rays),
               "prims_per_ray": prims / len(rays), "tree": "4-ary shadow tree" if st["wide_shadow_rays"] else "reference",
               "simd_eff": steps / max(1, st["wave_node_iters"] * 64), "spill": st["stack_spills"] / max(1, st["stack_pushes"])}
        for w in args.waves.split(","):
            os.environ["DRT_TRACE_WAVES"] = w
            ms = []
            for _ in range(args.reps):
                fn(rays)
                ms.append(r.trace_stats()["kernel_ms"])
            best = min(ms)
            rec[f"w{w}"] = {"ms": round(best, 3), "Mrays_s": round(len(rays) / best / 1e3, 1),
                            "Gsteps_s": round(steps / best / 1e6, 2)}
        out["sets"][name] = rec
        print(name, json.dumps(rec), flush=True)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
