"""Search for the survey's synthetic-scene generator.

The survey measured the reference's BVH on its 100k / 1M-triangle soups at 118 983 / 1 187 635 nodes
(SURVEY.md §6), but did not commit its generator; §8d gives only its spec.  The product's
generator (bench.synthetic_triangles) builds 118 991 nodes at 100k.  This script enumerates the spec's
open choices — draw order, the float32 rounding point, the P3F text precision the scene was written with
(the reference parses the text back), and the floor's diagonal and place in the object list — builds each
variant's BVH with the host library (the reference's exact tree, tests/test_host_library.py) and prints
the node counts.  CPU only.

    python tools/generator_search.py [--n 100000] [--target 118983]
"""
import argparse
import itertools
import json
import sys
from pathlib import Path

import numpy as np

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import distributionraytracer_amd as drt  # noqa: E402

FLOORS = {
    "diag_a": np.array([[-4, -4, -1.2, 4, -4, -1.2, 4, 4, -1.2], [-4, -4, -1.2, 4, 4, -1.2, -4, 4, -1.2]]),
    "diag_b": np.array([[-4, -4, -1.2, 4, -4, -1.2, -4, 4, -1.2], [4, -4, -1.2, 4, 4, -1.2, -4, 4, -1.2]]),
}


def soup(n, order, sum32, hmode, seed=1):
    rng = np.random.default_rng(seed)
    h = n ** (-1.0 / 3.0) if hmode == "pow" else 1.0 / np.cbrt(n)
    if order == "c_then_off":
        c = rng.uniform(-1.0, 1.0, size=(n, 1, 3))
        off = rng.uniform(-h, h, size=(n, 3, 3))
    elif order == "off_then_c":
        off = rng.uniform(-h, h, size=(n, 3, 3))
        c = rng.uniform(-1.0, 1.0, size=(n, 1, 3))
    elif order == "interleaved":
        a = rng.uniform(0.0, 1.0, size=(n, 12))
        c = (-1.0 + 2.0 * a[:, :3]).reshape(n, 1, 3)
        off = (-h + 2.0 * h * a[:, 3:]).reshape(n, 3, 3)
    elif order == "random_scaled":
        c = (rng.random((n, 1, 3)) * 2.0 - 1.0)
        off = (rng.random((n, 3, 3)) * 2.0 - 1.0) * h
    else:
        raise ValueError(order)
    if sum32:
        v = c.astype(np.float32) + off.astype(np.float32)
    else:
        v = (c + off).astype(np.float32)
    return v.reshape(n, 9)


def as_text(v, fmt):
    """The floats the reference reads back from P3F text written with `fmt` (None: exact float32)."""
    if fmt is None:
        return v.astype(np.float32)
    return np.array([float(fmt % x) for x in v.astype(np.float64).ravel()], np.float64).astype(np.float32).reshape(v.shape)


def nodes_of(tris):
    s = drt.Scene()
    s.set_accel("bvh")
    s.add_material((1, 0.9, 0.7), 0.5, (1, 1, 1), 0.5, 30.0827, 0, 1)
    s.add_triangles(tris)
    s.build()
    return s.info().bvh_nodes


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=100000)
    ap.add_argument("--target", type=int, default=118983)
    a = ap.parse_args()
    rows = []
    for order, sum32, hmode, fmt, floor, first in itertools.product(
            ("c_then_off", "off_then_c", "interleaved", "random_scaled"), (False, True), ("pow",),
            (None, "%.6f", "%.5f", "%.4f", "%g", "%.7g", "%.8g"), ("diag_a", "diag_b"), (False, True)):
        v = as_text(soup(a.n, order, sum32, hmode), fmt)
        fl = FLOORS[floor].astype(np.float32)
        tris = np.concatenate([fl, v]) if first else np.concatenate([v, fl])
        n = nodes_of(tris)
        row = dict(order=order, sum32=sum32, h=hmode, fmt=fmt, floor=floor, floor_first=first, nodes=n,
                   match=n == a.target)
        rows.append(row)
        print(json.dumps(row), flush=True)
    hits = [r for r in rows if r["match"]]
    print(json.dumps({"n": a.n, "target": a.target, "variants": len(rows), "matches": len(hits),
                      "node_counts": sorted({r["nodes"] for r in rows})}))


if __name__ == "__main__":
    main()
