"""The C++ drop-in (base::TraceScene & co., host/fs_host.h) used exactly like
the reference's main.cpp: N TraceScene calls == one N-spp render == oracle."""
import os
import subprocess

import numpy as np
import pytest

import fsamd
import oracle_py
import scenes
from conftest import ROOT, load_scene

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name,W,H,N", [("c2", 64, 40, 6), ("c4", 48, 32, 3)])
def test_trace_scene_loop_matches_oracle(name, W, H, N, scene_dir, tmp_path):
    """C4's 1 M-face mesh takes the device BVH build inside TraceScene."""
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "examples")], check=True)
    path = scenes.write(name, os.path.join(scene_dir, f"{name}_dropin"))
    ppm, f32 = str(tmp_path / "out.ppm"), str(tmp_path / "out.f32")
    subprocess.run([os.path.join(ROOT, "examples", "trace_scene"), path, str(W), str(H), str(N), ppm, f32],
                   check=True, timeout=300)
    color = np.fromfile(f32, np.float32).reshape(H, W, 3)
    s = load_scene(name, scene_dir)
    ref = oracle_py.Scene(s.desc_ptr()).render(s.camera(0), fsamd.render_params(W, H, N), threads=8)
    np.testing.assert_array_equal(color, ref.color)
    raw = open(ppm, "rb").read()
    img = np.frombuffer(raw[raw.index(b"255\n") + 4:], np.uint8).reshape(H, W, 3)
    np.testing.assert_array_equal(img[::-1], ref.display)
