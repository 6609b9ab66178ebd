"""Build tests/golden/shipped_scenes.npz: the reference's shipped P3D scenes as DATA fixtures.

The scenes (DistributionRayTracer/P3D_Scenes/*.p3f) are the reference's test inputs.  The GPU
box has no /root/reference, so the parity tests read them from this fixture instead:

  <name>/head   the scene text up to its `mesh` command (or all of it), as bytes
  mesh/dragon   the 50 000-vertex / 100 000-face mesh block shared by dragon, assignment1 and
                dragon_assignment1 (byte-identical in all three files), zlib-compressed
  sky/<dir>     the six cube faces of skybox, skybox1, skybox2 (right..back), decoded with PIL,
                rows bottom-up (IL_ORIGIN_LOWER_LEFT, scene.cpp:345), downsampled (nearest) to
                SKY x SKY so the fixture stays small; both the HIP path and the oracle are fed
                the same bytes

Run here, where the reference checkout exists:  python tests/golden/make_shipped_scenes.py
Nothing of the reference's code is read or stored; ajax.p3f is absent upstream
(.MISSING_LARGE_BLOBS).
"""
from __future__ import annotations

import hashlib
import zlib
from pathlib import Path

import numpy as np

REF = Path("/root/reference/DistributionRayTracer")
OUT = Path(__file__).resolve().parent / "shipped_scenes.npz"
SCENES = ["balls_low", "dof", "motion", "teste", "balls_box", "balls_high", "blueDiamond", "dragon",
          "assignment1", "dragon_assignment1"]
FACES = ("right", "left", "top", "bottom", "front", "back")
SKY = 64


def main():
    from PIL import Image

    arrs = {}
    mesh = None
    for name in SCENES:
        raw = (REF / "P3D_Scenes" / f"{name}.p3f").read_bytes()
        lines = raw.split(b"\n")
        cut = next((i for i, l in enumerate(lines) if l.split()[:1] == [b"mesh"]), None)
        if cut is not None and name in ("dragon", "assignment1", "dragon_assignment1"):
            head = b"\n".join(lines[:cut]) + b"\n"
            tail = b"\n".join(lines[cut:])
            if mesh is None:
                mesh = tail
            assert tail == mesh, f"{name}: mesh block differs"
            arrs[f"{name}/mesh"] = np.frombuffer(b"dragon", np.uint8)
        else:
            head = raw
        arrs[f"{name}/head"] = np.frombuffer(head, np.uint8)
        arrs[f"{name}/sha1"] = np.frombuffer(hashlib.sha1(raw).hexdigest().encode(), np.uint8)
    arrs["mesh/dragon"] = np.frombuffer(zlib.compress(mesh, 9), np.uint8)
    for d in ("skybox", "skybox1", "skybox2"):
        for f in FACES:
            im = Image.open(REF / d / f"{f}.jpg").convert("RGB").resize((SKY, SKY), Image.NEAREST)
            arrs[f"sky/{d}/{f}"] = np.asarray(im, np.uint8)[::-1].copy()
    np.savez_compressed(OUT, **arrs)
    print(OUT, OUT.stat().st_size, "bytes")


if __name__ == "__main__":
    main()
