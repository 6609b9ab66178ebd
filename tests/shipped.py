"""The reference's shipped P3D scenes, from the data fixture tests/golden/shipped_scenes.npz
(made by tests/golden/make_shipped_scenes.py), with optional overrides of single P3F commands
(resolution, spp, accel) for reduced-size parity runs."""
from __future__ import annotations

import re
import zlib
from functools import lru_cache
from pathlib import Path

import numpy as np

FIXTURE = Path(__file__).resolve().parent / "golden" / "shipped_scenes.npz"
FACES = ("right", "left", "top", "bottom", "front", "back")


@lru_cache(maxsize=1)
def _npz():
    return dict(np.load(FIXTURE))


def names():
    return sorted(k.split("/")[0] for k in _npz() if k.endswith("/head"))


def text(name, res=None, spp=None, accel=None) -> bytes:
    z = _npz()
    head = z[f"{name}/head"].tobytes()
    if res is not None:
        head, n = re.subn(rb"(?m)^resolution[ \t]+\d+[ \t]+\d+", b"resolution %d %d" % tuple(res), head)
        assert n == 1, name
    if spp is not None:
        head, n = re.subn(rb"(?m)^spp[ \t]+\d+", b"spp %d" % spp, head)
        assert n == 1, name
    if accel is not None:
        head, n = re.subn(rb"(?m)^accel[ \t]+\w+", b"accel " + accel.encode(), head)
        assert n == 1, name
    if f"{name}/mesh" in z:
        head += zlib.decompress(z["mesh/" + z[f"{name}/mesh"].tobytes().decode()].tobytes())
    return head


def env(name):
    m = re.search(rb"(?m)^env[ \t]+(\S+)", _npz()[f"{name}/head"].tobytes())
    return m.group(1).decode() if m else None


def skybox_faces(name):
    """The scene's six cube faces (bottom-up RGB8, downsampled), or None without `env`."""
    e = env(name)
    if e is None:
        return None
    z = _npz()
    return [z[f"sky/{e}/{f}"] for f in FACES]


def write(tmp_path, name, **over):
    p = Path(tmp_path) / f"{name}.p3f"
    p.write_bytes(text(name, **over))
    return p
