"""The Grid headline's shadow queries on the Grid scene's shadow tree (round 6): one stats frame with
the tree (DRT_GRID_SHADOW_TREE=2) and one on the walk — queries, tree work, certificates tried, queries
left to the Grid walk — as one JSON line."""
import json
import os
import sys
import types
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
import bench  # noqa: E402
import distributionraytracer_amd as drt  # noqa: E402

spp = int(sys.argv[1]) if len(sys.argv) > 1 else 64
args = types.SimpleNamespace(scene="synthetic", res=512, spp=spp)
ext = {"aperture": 0.0, "focal": 1.0, "accel": "grid", "ks": 0.5}
s = bench.make_scene(drt, args, bench.synthetic_triangles(1_000_000, 1), ext)
s.build()
r = drt.Renderer(0)
r.upload(s)
out = {"spp": spp}
for mode in ("2", "0"):
    os.environ["DRT_GRID_SHADOW_TREE"] = mode
    r.render(seed=7, stats=True)
    st = r.stats()
    out["tree" if mode == "2" else "walk"] = {k: st[k] for k in ("samples", "shadow_rays", "shadow_leaf", "shadow_prims",
                                                                "wide_shadow_rays", "wide_inner", "wide_leaf",
                                                                "wide_prims", "wide_verify", "wide_grid_walks")}
t = out["tree"]
out["grid_walk_frac"] = t["wide_grid_walks"] / max(1, t["shadow_rays"])
out["certified_frac_of_hits"] = 1 - t["wide_grid_walks"] / max(1, t["wide_verify"])
print(json.dumps(out))
r.close()
