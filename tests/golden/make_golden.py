"""Regenerates the golden fixtures of tests/golden from the ORACLE.

The reference cannot be built in this image (math/base.h:37-51 needs
<windows.h>/<TargetConditionals.h>), so these vectors come from the oracle's
restatement; they pin the oracle and the GPU path against regressions. The
reference-produced values recorded in SURVEY.md live in reference_probes.json
and are checked separately (tests/test_oracle.py).

    python tests/golden/make_golden.py
"""
import ctypes as C
import hashlib
import json
import os
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import fsamd  # noqa: E402
import oracle_py  # noqa: E402
import scenes  # noqa: E402

SEED = 521288629
IMAGES = {"c1": (32, 32, 8), "c2": (48, 32, 8)}


def rng_vectors():
    L = oracle_py.lib()
    s = C.c_uint64(SEED)
    ints = [L.oracle_random_integer(C.byref(s)) for _ in range(64)]
    s = C.c_uint64(SEED)
    floats = [float(np.float32(L.oracle_random_float(C.byref(s)))) for _ in range(16)]
    s = C.c_uint64(SEED)
    ranges = [int(L.oracle_random_integer_range(C.byref(s), 0, 32767)) for _ in range(16)]
    seeds = [int(L.oracle_pixel_seed(p, k, 0)) for p, k in ((0, 0), (1, 0), (0, 1), (123456, 1023))]
    return {"seed": SEED, "random_integer": [str(v) for v in ints], "random_float": floats,
            "random_integer_range_0_32767": ranges,
            "pixel_seed": [str(v) for v in seeds]}


def table_vectors():
    out = {}
    for pre in range(1, 9):
        t = np.zeros((32768, 3), np.float32)
        oracle_py.lib().oracle_normal_table(SEED, pre, 32768, oracle_py.fptr(t)[1])
        out[str(pre)] = {"sha256": hashlib.sha256(t.tobytes()).hexdigest(),
                         "first": t[:4].tolist(), "last": t[-4:].tolist()}
    return out


def main():
    json.dump(rng_vectors(), open(os.path.join(HERE, "rng.json"), "w"), indent=1)
    json.dump(table_vectors(), open(os.path.join(HERE, "normal_table.json"), "w"), indent=1)
    d = tempfile.mkdtemp()
    for name, (W, H, spp) in IMAGES.items():
        path = scenes.write(name, os.path.join(d, name))
        fsamd.reset_main_rng()
        s = fsamd.HostScene.load(path)
        fsamd.initialize_materials()
        o = oracle_py.Scene(s.desc_ptr())
        f = o.render(s.camera(0), fsamd.render_params(W, H, spp), threads=8)
        np.savez_compressed(os.path.join(HERE, f"{name}_{W}x{H}x{spp}.npz"), color=f.color, count=f.count,
                            display=f.display, normal=f.normal, depth=f.depth, material=f.material)
    print("golden fixtures written to", HERE)


if __name__ == "__main__":
    main()
