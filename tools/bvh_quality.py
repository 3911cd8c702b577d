"""BVH tree quality per mesh (fs_bvh_quality: SAH cost, sibling overlap per
level, counts, depth) of the bench scenes under fs_options build settings.
usage: python tools/bvh_quality.py c3,c4 [variant ...]   (variants as perf_ab.py)"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import fsamd  # noqa: E402
import scenes  # noqa: E402

names = sys.argv[1].split(",")
variants = sys.argv[2:] or ["default"]
for name in names:
    p = scenes.write(name, os.path.join("/tmp", "fs_bvhq", name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    for v in variants:
        q = fsamd.bvh_quality(s.desc_ptr(), **fsamd.parse_variant(v))
        for m in q:
            lv = m.pop("overlap_per_level")
            m["overlap_levels_0_8"] = [round(x, 3) for x in lv[:9]]
            print(name, v, json.dumps(m), flush=True)
