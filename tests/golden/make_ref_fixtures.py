#!/usr/bin/env python3
"""Generate tests/golden/ref_meshes.json from the REFERENCE's own readers (oracle/_ref:
tinyobjloader and stb_image compiled unmodified from /root/reference; run in the build
container, which has the reference tree).  Pins, for the GPU box where the reference is absent:

  meshes.<name>: tinyobj::LoadObj + Scene::LoadModel's triangle loop on assets/<name>.obj --
                 vertex / triangle counts and sha256 of the triangles' float32 vertex bits in
                 primitive-id order (template/scene.h:156-201); the bundled .rtmesh files must
                 hash to these (tests/test_ref_io.py);
  images.<name>: stbi_load + Surface::LoadImage on assets/<name>.png -- size, channels and
                 sha256 of the 0x00RRGGBB texels (template/template.cpp:1579-1601).

usage: python tests/golden/make_ref_fixtures.py"""
import hashlib
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import refio  # noqa: E402

ASSETS = os.path.join(refio.REFERENCE, "assets")


def main():
    if not refio.available():
        sys.exit("the reference tree is not here: run this in the build container")
    out = {"source": "oracle/_ref/libref_io.so: template/tiny_obj_loader.h + lib/stb_image.h from /root/reference, "
                     "unmodified (oracle/ref_io.cpp)", "meshes": {}, "images": {}}
    for name in ("teapot", "mig29", "Shiba", "glider"):
        V, F = refio.load_model(os.path.join(ASSETS, name + ".obj"))
        out["meshes"][name] = {"vertices": int(len(V)), "triangles": int(len(F)),
                               "vertices_sha256": hashlib.sha256(np.ascontiguousarray(V, np.float32).tobytes()).hexdigest(),
                               "triangles_sha256": hashlib.sha256(np.ascontiguousarray(V[F], np.float32).tobytes()).hexdigest()}
    for name in ("earth", "logo", "font"):
        px, n = refio.load_image(os.path.join(ASSETS, name + ".png"))
        out["images"][name] = {"width": int(px.shape[1]), "height": int(px.shape[0]), "channels": int(n),
                               "texels_sha256": hashlib.sha256(np.ascontiguousarray(px, np.uint32).tobytes()).hexdigest()}
    with open(os.path.join(HERE, "ref_meshes.json"), "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
