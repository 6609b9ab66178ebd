"""Synthetic P3F scene generators shared by the oracle, parity and bench code paths.

Scenes are emitted as P3F text (the reference's own format, scene.cpp:474-740) so the oracle
and the product parse byte-identical inputs.  Floats are written with the shortest repr that
round-trips through strtof, so every coordinate is exactly the float32 the generator made.
"""
from __future__ import annotations

import numpy as np


def ff(x) -> str:
    return np.format_float_positional(np.float32(x), unique=True, trim="-")


def vec(v) -> str:
    return " ".join(ff(c) for c in v)


BALLS_LOW_CAMERA = dict(eye=(2.1, 1.3, 1.7), at=(0, 0, 0), up=(0, 0, 1), angle=45, hither=0.01)


def header(res=(64, 64), spp=0, accel="bvh", bclr=(0.078, 0.361, 0.753), camera=None, aperture=0.0, focal=1.0,
           env=None):
    cam = dict(BALLS_LOW_CAMERA)
    if camera:
        cam.update(camera)
    lines = [f"accel {accel}", f"spp {spp}", f"bclr {vec(bclr)}"]
    if env:
        lines.append(f"env {env}")
    lines += ["camera", f"eye {vec(cam['eye'])}", f"at {vec(cam['at'])}", f"up {vec(cam['up'])}",
              f"angle {ff(cam['angle'])}", f"hither {ff(cam['hither'])}", f"resolution {res[0]} {res[1]}",
              f"aperture {ff(aperture)}", f"focal {ff(focal)}"]
    return lines


def mesh_lines(tris: np.ndarray):
    tris = np.asarray(tris, np.float32).reshape(-1, 3, 3)
    n = len(tris)
    out = [f"mesh {3 * n} {n}"]
    out += [vec(v) for v in tris.reshape(-1, 3)]
    out += [f"{3 * i + 1} {3 * i + 2} {3 * i + 3}" for i in range(n)]
    return out


def synthetic_triangles(n, seed=1):
    """centres U[-1,1]^3, vertices c + U[-h,h]^3, h = n^(-1/3), float32."""
    rng = np.random.default_rng(seed)
    h = n ** (-1.0 / 3.0)
    c = rng.uniform(-1.0, 1.0, size=(n, 1, 3))
    v = c + rng.uniform(-h, h, size=(n, 3, 3))
    return v.astype(np.float32).reshape(n, 9)


def survey_triangles(n, seed=1):
    """The survey's own soup, reconstructed (round 6, tools/generator_search.py): the §8d spec with each
    vertex the float32 sum c + offset of float32-rounded draws, written to the P3F text with 7 significant
    digits (%.7g) and parsed back by the reference's loader.  At 100k triangles (+ floor) the reference's
    BVH build then has the 118 983 nodes the survey measured; at 1M it has 1 187 633 against
    the survey's 1 187 635 (no variant tried matched both)."""
    rng = np.random.default_rng(seed)
    h = n ** (-1.0 / 3.0)
    c = rng.uniform(-1.0, 1.0, size=(n, 1, 3)).astype(np.float32)
    v = (c + rng.uniform(-h, h, size=(n, 3, 3)).astype(np.float32)).reshape(-1)
    return np.array([float("%.7g" % x) for x in v.tolist()], np.float64).astype(np.float32).reshape(n, 9)


FLOOR = np.array([[-4, -4, -1.2, 4, -4, -1.2, 4, 4, -1.2], [-4, -4, -1.2, 4, 4, -1.2, -4, 4, -1.2]], np.float32)
SYNTH_MAT = "mat 1 0.9 0.7 0.5 1 1 1 0.5 30.0827 0 1"
SYNTH_LIGHTS = ["light quad 4 3 2 1 1 1 4 2 2 3 3 2 16", "light punctual -3 1 5 1 1 1"]


def write_synthetic_p3f(path, n_tris, res=(512, 512), spp=64, accel="bvh", seed=1, aperture=0.0, focal=1.0):
    """synthetic_scene_text written fast for large n (np.savetxt, '%.9g' floats: every float32
    round-trips through strtof exactly, so the parsed scene is the same).  Returns the path."""
    tris = np.concatenate([synthetic_triangles(n_tris, seed), FLOOR]).reshape(-1, 3, 3)
    n = len(tris)
    lines = header(res=res, spp=spp, accel=accel, aperture=aperture, focal=focal) + SYNTH_LIGHTS + [SYNTH_MAT]
    with open(path, "w") as f:
        f.write("\n".join(lines) + f"\nmesh {3 * n} {n}\n")
        np.savetxt(f, tris.reshape(-1, 3), fmt="%.9g")
        np.savetxt(f, np.arange(1, 3 * n + 1, dtype=np.int64).reshape(n, 3), fmt="%d")
    return path


def synthetic_scene_text(n_tris, res=(512, 512), spp=64, accel="bvh", seed=1, aperture=0.0, focal=1.0):
    """The §8d benchmark scene: triangle soup + floor, one quad and one point light."""
    lines = header(res=res, spp=spp, accel=accel, aperture=aperture, focal=focal)
    lines += SYNTH_LIGHTS
    lines.append(SYNTH_MAT)
    lines += mesh_lines(np.concatenate([synthetic_triangles(n_tris, seed), FLOOR]))
    return "\n".join(lines) + "\n"


def mixed_scene_text(res=(48, 40), spp=4, accel="bvh", seed=7, n_tris=300, aperture=0.0, focal=1.0, quad=True,
                     glass=True, bclr=(0.078, 0.361, 0.753), cluster=0, env=None):
    """Spheres (mirror + glass), boxes, planes, triangles, quad + point lights.

    cluster > 0 adds `cluster` concentric spheres and `cluster` triangles spun about one
    centroid: coincident centroids leave the SAH no split (bvh.cpp:187-189), so the BVH gets
    oversized leaves (>= 31 objects, the layout's count-31 escape)."""
    rng = np.random.default_rng(seed)
    lines = header(res=res, spp=spp, accel=accel, aperture=aperture, focal=focal, bclr=bclr, env=env)
    if quad:
        lines.append("light quad 4 3 2 1 1 1 4 2 2 3 3 2 4")
    lines.append("light punctual -3 1 5 1 1 1")
    lines.append("light punctual 1 -4 4 1 1 1")
    lines.append("mat 1 0.75 0.33 1 1 1 0.8 0 10 0 1")
    lines.append("pl 12 12 -0.5 -12 12 -0.5 -12 -12 -0.5")
    lines.append("mat 1 0.9 0.7 0.5 1 1 1 0.5 30.0827 0 1")
    for _ in range(8):
        c = rng.uniform(-0.8, 0.8, 3)
        lines.append(f"s {vec(c)} {ff(rng.uniform(0.05, 0.3))}")
    if glass:
        lines.append("mat 0 0.5 0 0 1 1 1 0.2 30.1 1 1.15")
        lines.append(f"s {vec((0.3, -0.2, 0.1))} {ff(0.25)}")
        lines.append("mat 0.8 0.8 0.8 0 1 1 1 0.2 20 1 1.35")
        lines.append(f"s {vec((-0.4, 0.4, 0.2))} {ff(0.2)}")
    lines.append("mat 0.5 0.4 0.5 0 1.0 0.71 0.29 0.9 200 0 1")
    lines.append(f"box {vec((0.1, 0.1, -0.4))} {vec((0.5, 0.6, 0.0))}")
    lines.append("mat 0.6667 0.996 0.8745 0.75 1 1 1 0.25 100 0 1")
    t = synthetic_triangles(n_tris, seed) * 0.6
    if cluster:
        lines.append("mat 0.3 0.6 0.9 0.6 1 1 1 0.4 40 0 1")
        for k in range(cluster):
            lines.append(f"s {vec((-0.5, -0.5, 0.3))} {ff(0.05 + 0.004 * k)}")
        a = np.linspace(0.0, np.pi, cluster, endpoint=False)[:, None]
        c = np.array([0.55, -0.45, 0.35])
        u = np.concatenate([np.cos(a), np.sin(a), 0 * a], 1) * 0.2
        w = np.concatenate([-np.sin(a), np.cos(a), 0 * a], 1) * 0.1
        # vertices c + u, c - u/2 + w*sqrt3, c - u/2 - w*sqrt3 ... centroid exactly c in exact math;
        # float rounding may split a few, the rest stay together
        spun = np.stack([c + u, c - u / 2 + w, c - u / 2 - w], 1).reshape(-1, 9)
        t = np.concatenate([t, spun.astype(np.float32)])
    lines += mesh_lines(t)
    return "\n".join(lines) + "\n"


def random_rays(n, seed=3, origin_box=1.5, toward_origin=True):
    rng = np.random.default_rng(seed)
    o = rng.uniform(-origin_box, origin_box, (n, 3))
    if toward_origin:
        d = rng.uniform(-0.5, 0.5, (n, 3)) - o
    else:
        d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    r = np.concatenate([o, d], axis=1).astype(np.float32)
    # a few axis-aligned directions: 1.0/0 = inf slabs, NaN products on boundaries
    k = max(1, n // 16)
    r[:k, 3:] = 0.0
    r[:k, 3 + (np.arange(k) % 3)] = np.where(np.arange(k) % 2, 1.0, -1.0)
    return r


def write(tmp_path, name, text):
    p = tmp_path / name
    p.write_text(text)
    return p


def balls_low_text(res=(512, 512), spp=16, accel="none"):
    """The geometry, lights and materials of P3D_Scenes/balls_low.p3f,
    with resolution / spp / accel as parameters."""
    lines = header(res=res, spp=spp, accel=accel)
    lines += ["light quad 4 3 2 1 1 1 4 2 2 3 3 2 16", "light quad 1 -4 4 1 1 1 0 -4 4 1 -3 4 16",
              "light punctual -3 1 5 1 1 1",
              "mat 1 0.75 0.33 1 1 1 0.8 0 10 0 1", "pl 12 12 -0.5 -12 12 -0.5 -12 -12 -0.5",
              "mat 1 0.9 0.7 0.5 1 1 1 0.5 30.0827 0 1", "s 0 0 0 0.5"]
    a, b, c, d, e = "0.272166", "0.643951", "0.172546", "0.371785", "0.0996195"
    f, z, r = "0.471405", "1.11022e-16", "0.166667"
    for x, y, zz in ((a, a, "0.544331"), (b, c, z), (c, b, z), ("-" + d, e, "0.544331"), ("-" + f, f, z),
                     ("-" + b, "-" + c, z), (e, "-" + d, "0.544331"), ("-" + c, "-" + b, z), (f, "-" + f, z)):
        lines.append(f"s {x} {y} {zz} {r}")
    return "\n".join(lines) + "\n"


def set_accel(text, accel):
    """The same P3F text with its `accel` command set to `accel` (added if absent)."""
    lines = text.split("\n")
    for i, l in enumerate(lines):
        if l.split()[:1] == ["accel"]:
            lines[i] = f"accel {accel}"
            return "\n".join(lines)
    return f"accel {accel}\n" + text
