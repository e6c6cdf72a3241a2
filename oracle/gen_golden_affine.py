"""Golden vectors for reverse_affine_map, made by running the REFERENCE's own code.

TEST INFRASTRUCTURE, run in the build container only (needs /root/reference):
    python oracle/gen_golden_affine.py        -> tests/golden/affine_maps.npz

Executed from where they lie (ast-extracted: the file's torchvision / cv2 imports are skipped):
``src/Utils/transformations.py`` ``reverse_affine_map`` (:7-77), ``kpt_affine`` (:131-135),
``get_transform`` (:142-167), ``get_affine_transform`` (:170-213), ``get_multi_scale_size`` (:216-238).
OpenCV is absent from this image: ``cv2.getAffineTransform`` is stubbed by its documented algorithm
(the 6 x 6 system of the three point correspondences solved in float64), so the solve itself is
parity unpinned; everything around it is the reference's code. numpy >= 1.24 dropped the ``np.float``
alias the reference uses: the extracted functions see a namespace with it restored.
"""
import ast
import os
import sys
import types

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle.ref_shims import REF_SRC  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "affine_maps.npz")
NAMES = ["reverse_affine_map", "kpt_affine", "get_transform", "get_affine_transform", "get_multi_scale_size"]


def get_affine_transform_cv2(src, dst):
    """cv::getAffineTransform: M (2 x 3, float64) with dst_i = M [src_i, 1] from three float32 pairs."""
    s, d = np.float32(src).astype(np.float64), np.float32(dst).astype(np.float64)
    a = np.zeros((6, 6))
    for i in range(3):
        a[2 * i, :3] = [s[i, 0], s[i, 1], 1.0]
        a[2 * i + 1, 3:] = [s[i, 0], s[i, 1], 1.0]
    b = np.array([d[0, 0], d[0, 1], d[1, 0], d[1, 1], d[2, 0], d[2, 1]])
    return np.linalg.solve(a, b).reshape(2, 3)


def load_reference():
    npc = types.ModuleType("numpy_compat")
    npc.__dict__.update(np.__dict__)
    npc.float, npc.int = float, int
    ns = {"np": npc, "cv2": types.SimpleNamespace(getAffineTransform=get_affine_transform_cv2)}
    path = os.path.join(REF_SRC, "Utils", "transformations.py")
    tree = ast.parse(open(path).read(), filename=path)
    body = [n for n in tree.body if isinstance(n, ast.FunctionDef) and n.name in NAMES]
    assert {n.name for n in body} == set(NAMES)
    exec(compile(ast.Module(body=body, type_ignores=[]), path, "exec"), ns)
    return ns


CASES = [   # (width, height, input_size, scaling_type, min_scale)
    (640, 480, 512, "short", 1.0), (427, 640, 512, "short", 1.0), (500, 375, 640, "short", 1.0),
    (333, 500, 640, "short_with_resize", 0.5), (640, 427, 512, "short_with_resize", 1.0),
    (612, 612, 640, "short", 1.0), (640, 480, 512, "long", 1.0), (375, 500, 512, "long_with_multiscale", 1.0),
]


def main():
    ref = load_reference()
    rng = np.random.default_rng(5)
    out = {}
    for c, (w, h, size, kind, ms) in enumerate(CASES):
        kp = np.concatenate([rng.uniform(0, 320, (4, 17, 2)), rng.uniform(0, 1, (4, 17, 1))], 2)
        got = ref["reverse_affine_map"](kp.copy(), (w, h), size, scaling_type=kind, min_scale=ms)
        out[f"in_{c}"] = kp
        out[f"out_{c}"] = got
    out["cases"] = np.array([f"{w},{h},{s},{k},{m}" for w, h, s, k, m in CASES])
    np.savez(OUT, **out)
    print(f"wrote {OUT}: {len(CASES)} cases")


if __name__ == "__main__":
    main()
