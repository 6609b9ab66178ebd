"""GPU parity of the 4-ary shadow tree (drt_layout.hpp, DESIGN.md §4 "shadow tree").

BVH::Traverse(Ray&) (bvh.cpp:316-391) returns true iff some primitive of a leaf whose box the ray
hits (every ancestor box is then hit too: a node's box is the union of its objects' boxes, and the
slab values are monotone in the planes) has a hit with t <= |Ls| + EPSILON.  That boolean does not
depend on the visit order, so finite shadow rays walk a 4-ary tree collapsed from the reference's
tree, whose quantised child boxes contain the reference boxes, and an in-range hit counts only once
its leaf's exact reference box is hit.  These tests hold the answer to the reference's: the golden
vectors (test_gpu_parity.py), the reference-order traversal on >= 10^7 frame-like shadow rays of
the 1M-triangle headline scene, the oracle, and the edge cases of the slab test.
"""
import numpy as np
import pytest

from tests import scenegen as sg

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def drt():
    import distributionraytracer_amd as d

    return d


@pytest.fixture(scope="module")
def renderer(drt):
    r = drt.Renderer(0)
    yield r
    r.close()


def primary_rays(scene, n, seed):
    """Camera::PrimaryRay (camera.h:74-83) through n random pixel positions (numpy, float32)."""
    c = scene.camera_frame()
    rng = np.random.default_rng(seed)
    px = rng.uniform(0, c.res_x, n).astype(np.float32)
    py = rng.uniform(0, c.res_y, n).astype(np.float32)
    u, v, w = (np.array(getattr(c, k), np.float32) for k in ("u", "v", "n"))
    a = (px / np.float32(c.res_x) - np.float32(0.5))[:, None]
    b = (py / np.float32(c.res_y) - np.float32(0.5))[:, None]
    d = u * np.float32(c.w) * a + v * np.float32(c.h) * b - w * np.float32(c.plane_dist)
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    o = np.broadcast_to(np.array(c.eye, np.float32), d.shape)
    return np.concatenate([o, d], axis=1).astype(np.float32)


def shadow_rays_from_hits(rays, t, nrm, obj, lights, rng):
    """rayTracing's shadow rays (main.cpp:386-422) from the hits of `rays`: origin hitPoint +
    N*1e-4 with N facing the ray, direction the unnormalised Ls towards each light point."""
    hit = obj >= 0
    o, d, t, nrm = rays[hit, :3], rays[hit, 3:], t[hit], nrm[hit]
    p = o + d * t[:, None]
    n = nrm / np.linalg.norm(nrm, axis=1, keepdims=True)
    n = np.where((np.sum(d * n, axis=1) < 0)[:, None], n, -n)
    so = (p + n * np.float32(1e-4)).astype(np.float32)
    out = []
    for lp in lights(len(so), rng):
        out.append(np.concatenate([so, (lp - so).astype(np.float32)], axis=1))
    return np.concatenate(out).astype(np.float32)


def bench_lights(n, rng):
    """bench.populate's lights: the quad (4,3,2)+s*(0,-1,0)+t*(-1,0,0) at random points, the point light."""
    s = rng.random((n, 2), dtype=np.float32)
    quad = np.array([4, 3, 2], np.float32) + s[:, :1] * np.array([0, -1, 0], np.float32) + \
        s[:, 1:] * np.array([-1, 0, 0], np.float32)
    for _ in range(3):  # light_spp-style extra quad samples
        s = rng.random((n, 2), dtype=np.float32)
        yield np.array([4, 3, 2], np.float32) + s[:, :1] * np.array([0, -1, 0], np.float32) + \
            s[:, 1:] * np.array([-1, 0, 0], np.float32)
    yield quad
    yield np.broadcast_to(np.array([-3, 1, 5], np.float32), (n, 3))


def trace_shadow_both(renderer, rays):
    """Occlusion on the shadow tree and on the reference's tree (reference visit order), with the
    traversal counts of each."""
    renderer.set_trace_stats(True)
    wide = renderer.trace_shadow(rays)
    st_w = renderer.trace_stats()
    renderer.set_trace_stats(True, reference_order=True)
    ref = renderer.trace_shadow(rays)
    st_r = renderer.trace_stats()
    renderer.set_trace_stats(False)
    return wide, ref, st_w, st_r


def test_shadow_tree_equals_reference_order_on_1e7_frame_shadow_rays(drt, renderer):
    """The headline scene (1M triangles + floor, bench.populate): 3 M primary rays, each hit with
    five light points (four on the quad, the point light), > 1e7 shadow rays.  Occlusion on the
    shadow tree equals the reference-order traversal bit for bit, with far fewer node visits."""
    import bench

    s = drt.Scene()
    bench.populate(s, bench.synthetic_triangles(1_000_000), 512, 64)
    s.build()
    renderer.upload(s)
    prim = primary_rays(s, 3_000_000, seed=5)
    t, nrm, obj = renderer.trace_closest(prim)
    rays = shadow_rays_from_hits(prim, t, nrm, obj, bench_lights, np.random.default_rng(6))
    assert len(rays) >= 10_000_000
    wide, ref, st_w, st_r = trace_shadow_both(renderer, rays)
    np.testing.assert_array_equal(wide, ref)
    assert 0.05 < wide.mean() < 0.95  # both answers occur
    # the few rays with a zero direction component keep the reference's tree (its slab NaN rules)
    assert len(rays) - 100 < st_w["wide_shadow_rays"] <= len(rays) and st_r["wide_shadow_rays"] == 0
    assert st_w["shadow_inner"] < 0.001 * st_r["shadow_inner"]
    # the point of the tree: fewer node records per query
    assert st_w["wide_inner"] < 0.75 * st_r["shadow_inner"], (st_w["wide_inner"], st_r["shadow_inner"])
    print(f"\n{len(rays)} shadow rays, occluded {wide.mean():.3f}: per query wide inner {st_w['wide_inner'] / len(rays):.2f} "
          f"leaf {st_w['wide_leaf'] / len(rays):.2f} prims {st_w['wide_prims'] / len(rays):.2f} verify "
          f"{st_w['wide_verify'] / len(rays):.3f} | reference inner {st_r['shadow_inner'] / len(rays):.2f} leaf "
          f"{st_r['shadow_leaf'] / len(rays):.2f} prims {st_r['shadow_prims'] / len(rays):.2f}")


@pytest.mark.parametrize("cluster", [0, 40])
def test_shadow_tree_matches_oracle_on_mixed_primitives(drt, oracle_mod, renderer, tmp_path, cluster):
    """Spheres, boxes, planes (whose default [-1,1]^3 box decides which rays see them inside the
    BVH, SURVEY Q7 — the case the exact leaf-box check exists for) and triangles; oversized leaves
    with cluster 40.  Random rays of random lengths, rays from inside boxes, and axis-parallel rays
    (a zero direction component: the reference's slab NaN rules, walked on the binary tree)."""
    p = sg.write(tmp_path, "s.p3f", sg.mixed_scene_text(accel="bvh", n_tris=300, cluster=cluster))
    a, b = drt.Scene.load_p3f(p), oracle_mod.Scene.load_p3f(p)
    renderer.upload(a)
    rng = np.random.default_rng(11)
    rays = sg.random_rays(60_000, seed=12).astype(np.float32)
    rays[:, 3:] *= rng.uniform(0.05, 8.0, (len(rays), 1)).astype(np.float32)  # ranges |Ls| + EPSILON
    rays[:5000, :3] = rng.uniform(-1.0, 1.0, (5000, 3))  # origins inside the plane's default box
    ax = rays[5000:8000]
    ax[np.arange(len(ax)), 3 + rng.integers(0, 3, len(ax))] = 0.0  # a zero direction component
    rays[8000:9000, 3:] = 0.0  # zero-length: NaN direction after normalisation
    wide, ref, st_w, st_r = trace_shadow_both(renderer, rays)
    np.testing.assert_array_equal(wide, ref)
    np.testing.assert_array_equal(wide, b.trace_shadow(rays))
    assert st_w["wide_shadow_rays"] > 0 and st_w["shadow_rays"] == len(rays)
    assert st_w["wide_shadow_rays"] < len(rays)  # the non-finite rays keep the reference's tree
