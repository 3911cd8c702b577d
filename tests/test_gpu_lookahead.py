"""The lookahead of small renders (fs_options.lookahead, ABI 9): a whole-frame
render of at most 4 spp that continues the previous call's sequence also traces
the next calls' samples in the background; those calls fold them. Frames must
be those of the plain loop, bit for bit against the oracle, whatever the caller
does between calls (camera change, frame reset, re-upload, another frame, a gap
in sample_base, a sequence dropped while its traces still run)."""
import numpy as np
import pytest

import fsamd
import oracle_py
from conftest import load_scene
from test_gpu_parity import assert_parity

pytestmark = pytest.mark.gpu

W, H = 96, 64


def planes(f):
    return {p: f.read(p) for p in range(6)}


def oracle_seq(desc, steps):
    """steps: (camera, spp, sample_base) in call order, into one frame."""
    o = oracle_py.Scene(desc)
    fr = None
    for cam, spp, base in steps:
        fr = o.render(cam, fsamd.render_params(W, H, spp, sample_base=base), frame=fr, threads=16)
    o.close()
    return fr


def gpu_seq(r, frame, steps, reset_at=()):
    folded = []
    for i, (cam, spp, base) in enumerate(steps):
        if i in reset_at:
            frame.reset()
        r.render(cam, frame, spp=spp, sample_base=base)
        folded.append(r.last_lookahead())
    return folded


@pytest.mark.parametrize("name,spp", [("c2", 1), ("c4", 1), ("c2", 3)])
def test_lookahead_loop_bit_exact(name, spp, scene_dir, gpu_renderer):
    """N calls of spp samples each (TraceScene's loop): the second call
    continues the first and starts the lookahead, every later call folds it,
    and the frame (colour, count, display and the last sample's normal / depth
    / material) equals the oracle's."""
    s = load_scene(name, scene_dir)
    cam = s.camera(0)
    gpu_renderer.upload(s)
    f = gpu_renderer.frame(W, H)
    steps = [(cam, spp, k * spp) for k in range(5)]
    folded = gpu_seq(gpu_renderer, f, steps)
    assert folded == [False, False, True, True, True]
    assert gpu_renderer.last_launches() == (1, spp)
    assert gpu_renderer.last_trace_ms() > 0
    out = planes(f)
    f.close()
    ref = oracle_seq(s.desc_ptr(), [(cam, 5 * spp, 0)])
    assert_parity(out, ref, exact=True)


def test_lookahead_discarded_when_the_call_changes(scene_dir, gpu_renderer):
    """A camera change, a skipped sample index and a lens camera between
    calls: a call that changes the camera traces anew (no fold, and starts no
    lookahead until the next call continues it); a skip of one sample index
    still finds the lookahead (24 calls ahead by default; with lookahead 1 it
    misses); a frame reset keeps it. Every frame is the oracle's for the same
    call sequence."""
    s = load_scene("c2", scene_dir)
    a = s.camera(0)
    b = fsamd.camera((2, 9, -30), (0, 10, 0), fov_y=44, aperture=0.0)
    lens = fsamd.camera((0, 10, -34), (0, 10, 0), fov_y=40, aperture=0.8, focal_depth=30)
    gpu_renderer.upload(s)
    f = gpu_renderer.frame(W, H)
    steps = [(a, 1, 0), (a, 1, 1), (b, 1, 2), (b, 1, 3), (b, 1, 5), (b, 1, 6), (lens, 1, 7), (lens, 1, 8)]
    folded = gpu_seq(gpu_renderer, f, steps)
    assert folded == [False, False, False, False, True, True, False, False]
    gpu_renderer.set_options(lookahead=1)  # depth 1: the skip misses
    more = [(a, 1, 9), (a, 1, 10), (a, 1, 11), (a, 1, 13), (a, 1, 14)]
    folded = gpu_seq(gpu_renderer, f, more)
    assert folded == [False, False, True, False, False]
    steps += more
    gpu_renderer.set_options(lookahead=2)
    out = planes(f)
    assert_parity(out, oracle_seq(s.desc_ptr(), steps), exact=True)
    # a reset between two calls of the same sequence: the fold goes into the reset frame
    steps2 = [(a, 1, 0), (a, 1, 1), (a, 1, 2)]
    folded = gpu_seq(gpu_renderer, f, steps2, reset_at=(2,))
    assert folded == [False, False, True]
    out = planes(f)
    f.close()
    assert_parity(out, oracle_seq(s.desc_ptr(), [(a, 1, 2)]), exact=True)


def test_lookahead_after_reupload_and_across_frames(scene_dir, gpu_renderer):
    """A re-upload drops the lookahead (it read the old scene); two frames fed
    alternately take each other's lookahead only when the call is the same,
    and both equal the plain loop with lookahead off."""
    s2 = load_scene("c2", scene_dir)
    cam = s2.camera(0)
    gpu_renderer.upload(s2)
    f = gpu_renderer.frame(W, H)
    gpu_renderer.render(cam, f, spp=1, sample_base=0)
    gpu_renderer.render(cam, f, spp=1, sample_base=1)  # starts a lookahead
    gpu_renderer.upload(s2)  # same scene, new upload: the pending traces are dropped
    gpu_renderer.render(cam, f, spp=1, sample_base=2)
    assert not gpu_renderer.last_lookahead()
    gpu_renderer.render(cam, f, spp=1, sample_base=3)
    assert not gpu_renderer.last_lookahead()
    gpu_renderer.render(cam, f, spp=1, sample_base=4)
    assert gpu_renderer.last_lookahead()
    out = planes(f)
    assert_parity(out, oracle_seq(s2.desc_ptr(), [(cam, 5, 0)]), exact=True)
    g = gpu_renderer.frame(W, H)
    f.reset()
    for k in range(3):  # f and g each get samples 0, 1, 2
        gpu_renderer.render(cam, f, spp=1, sample_base=k)
        gpu_renderer.render(cam, g, spp=1, sample_base=k)
    a, b = planes(f), planes(g)
    gpu_renderer.set_options(lookahead=0)
    h = gpu_renderer.frame(W, H)
    for k in range(3):
        gpu_renderer.render(cam, h, spp=1, sample_base=k)
        assert not gpu_renderer.last_lookahead()
    c = planes(h)
    for p in range(6):
        np.testing.assert_array_equal(a[p], c[p])
        np.testing.assert_array_equal(b[p], c[p])
    for fr in (f, g, h):
        fr.close()


def test_frame_map_is_the_plane(scene_dir, gpu_renderer):
    """fs_frame_map's page-locked copy equals fs_frame_read, plane by plane."""
    s = load_scene("c2", scene_dir)
    gpu_renderer.upload(s)
    f = gpu_renderer.frame(W, H)
    gpu_renderer.render(s.camera(0), f, spp=2)
    for p in range(6):
        np.testing.assert_array_equal(f.map(p), f.read(p))
    f.close()


def test_lookahead_full_width_fold_bit_exact(scene_dir, gpu_renderer):
    """A frame large enough for the one-lane-per-pixel fold of a lookahead
    call (fold_paths_lite, not the split fold of small frames): four calls,
    the last two folded from one lookahead launch of eight calls (traced with
    fewer waves per SIMD, bg_waves), every plane the oracle's."""
    s = load_scene("c2", scene_dir)
    cam = s.camera(0)
    gpu_renderer.upload(s)
    w, h = 1024, 960
    f = gpu_renderer.frame(w, h)
    folded = []
    for k in range(4):
        gpu_renderer.render(cam, f, spp=1, sample_base=k)
        folded.append(gpu_renderer.last_lookahead())
    assert folded == [False, False, True, True]
    out = planes(f)
    f.close()
    o = oracle_py.Scene(s.desc_ptr())
    ref = o.render(cam, fsamd.render_params(w, h, 4), threads=16)
    o.close()
    assert_parity(out, ref, exact=True)


def test_dropped_sequences_reuse_their_slots_bit_exact(scene_dir, gpu_renderer):
    """Sequences dropped while their background traces still run (C4, window
    24: the dropped launches' queues are cancelled on the context stream) and
    new sequences launched into the same slots at once, several times over:
    the folds of the new sequences read only their own traces, and the frame
    equals the oracle's for the same calls."""
    s = load_scene("c4", scene_dir)
    a = s.camera(0)
    b = fsamd.camera((2, 9, -30), (0, 10, 0), fov_y=44, aperture=0.0)
    gpu_renderer.upload(s)
    gpu_renderer.set_options(lookahead=24)
    f = gpu_renderer.frame(W, H)
    steps, folded = [], []
    for rnd in range(3):
        cam = (a, b)[rnd % 2]
        seq = [(cam, 1, k) for k in range(5)]
        f.reset()
        folded += gpu_seq(gpu_renderer, f, seq)
        steps = seq
    assert folded == [False, False, True, True, True] * 3
    out = planes(f)
    f.close()
    assert_parity(out, oracle_seq(s.desc_ptr(), steps), exact=True)
