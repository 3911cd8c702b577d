"""Times the oracle (CPU restatement, reference octree, row-band threads) in
this container on the configurations SURVEY.md §8(d) / Appendix A quote
reference rates and octree work counts for (8 threads), and prints the
oracle's own counts beside the survey's, so a rate ratio can be split into
"different scene" and "different machine":

  probe250 / probe1m  SURVEY Appendix A's probe: the C1 room + a 500 x 250 /
                      1000 x 500 UV-sphere blob (scenes.write_probe)
  c1                  C1 at 256 x 256
  c4                  the bench scene (blob + spheres + cuboid)

usage: python tools/cpu_calibration.py [threads] [names]"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"), os.path.join(ROOT, "oracle")]
import fsamd  # noqa: E402
import oracle_py  # noqa: E402
import scenes  # noqa: E402

# SURVEY.md §8(d) and Appendix A [probe]: reference Msamples/s on 8 threads, and
# the reference octree's segments per sample and triangle tests per segment
REF_RATE = {"c1": 0.73, "probe250": 0.180, "probe1m": 0.067, "c4": 0.067}
REF_COUNTS = {"c1": (5.1, 15.8), "probe250": (5.02, 137.0), "probe1m": (5.05, 451.0)}
# (name, W, H, spp, tile stride): about 5-10 s of oracle time each on 8 threads
CONFIGS = (("c1", 256, 256, 32, 1), ("probe250", 1920, 1080, 1, 2), ("probe1m", 1920, 1080, 1, 4),
           ("c4", 1920, 1080, 1, 4))


def main():
    threads = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    which = sys.argv[2].split(",") if len(sys.argv) > 2 else [c[0] for c in CONFIGS]
    for name, W, H, spp, stride in CONFIGS:
        if name not in which:
            continue
        d = f"/tmp/fs_calib/{name}"
        if name == "probe250":
            p = scenes.write_probe(d, nu=500, nv=250)
        elif name == "probe1m":
            p = scenes.write_probe(d, nu=1000, nv=500)
        else:
            p = scenes.write(name, d)
        fsamd.reset_main_rng()
        s = fsamd.HostScene.load(p)
        fsamd.initialize_materials()
        t = time.time()
        o = oracle_py.Scene(s.desc_ptr())
        build = time.time() - t
        prm = fsamd.render_params(W, H, spp, tile_stride=stride)
        t = time.perf_counter()
        f = o.render(s.camera(0), prm, threads=threads)
        dt = time.perf_counter() - t
        st = f.stats
        rate = st["samples"] / dt / 1e6
        seg = st["segments"] / max(st["samples"], 1)
        tri = st["tri_tests"] / max(st["segments"], 1)
        node = st["node_visits"] / max(st["segments"], 1)
        rs, rt = REF_COUNTS.get(name, (None, None))
        counts = f"segments/sample {seg:.2f} (survey {rs}), tri tests/segment {tri:.1f} (survey {rt}), " \
                 f"octree nodes/segment {node:.1f}"
        if rs:  # the rate per triangle test, which takes the scene's path lengths out of the ratio
            counts += f"; per triangle test x{(rate * seg * tri) / (REF_RATE[name] * rs * rt):.2f}"
        print(f"{name} {W}x{H}: {st['samples']} samples in {dt:.1f}s -> {rate:.3f} Msamples/s "
              f"(reference probe {REF_RATE[name]}; ratio {rate / REF_RATE[name]:.2f}); {counts}; "
              f"octree build {build:.1f}s", flush=True)
        o.close()


if __name__ == "__main__":
    main()
