"""Predicts multi-GPU strong scaling on one GPU: renders each rank's tile
share (tile_offset r, tile_stride N) of the bench frame in turn and reports
the slowest rank's render time per N (gather excluded).
usage: python tools/scaling_sim.py [scene] [spp] [Ns] [variants]
(variants: comma list of fs_options settings, e.g. "groups=1,default"; TS=<n> sets the tile size)"""
import os
import tempfile
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "final-stage-path-tracer-2-0_amd"))
import fsamd  # noqa: E402
import scenes  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "c4"
    spp = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
    ns = [int(v) for v in (sys.argv[3] if len(sys.argv) > 3 else "1,2,4,8").split(",")]
    variants = (sys.argv[4] if len(sys.argv) > 4 else "default").split(",")
    W, H = 1920, 1080
    p = scenes.write(name, os.path.join(tempfile.gettempdir(), "fs_scenes", name))
    fsamd.reset_main_rng()
    s = fsamd.HostScene.load(p)
    fsamd.initialize_materials()
    r = fsamd.Renderer(0)
    r.upload(s)
    cam = s.camera(0)
    f = r.frame(W, H)
    r.render(cam, f, spp=64)  # warm up (allocations, caches)
    for v in variants:
        opts = fsamd.parse_variant(v)
        ts = int(opts.pop("TS", 64))  # tile size (a render parameter, not an option)
        r.set_options(**fsamd.options_dict(fsamd.options(**opts)))
        base = None
        for n in ns:
            times, trace = [], []
            for rank in range(n):
                f.reset()
                r.render(cam, f, spp=spp, tile_offset=rank, tile_stride=n, tile_size=ts)
                times.append(r.last_render_ms())
                trace.append(r.last_trace_ms())  # the trace kernel's share; the rest is fold_paths
            launches = r.last_launches()
            worst = max(times)
            rate = W * H * spp / worst / 1e3
            base = base or rate
            print(f"{name} {v} N={n}: slowest rank {worst:.1f} ms (mean {sum(times)/n:.1f}), "
                  f"{rate:.0f} Msamples/s, efficiency {rate / base / n:.3f}, launches/rank {launches}; "
                  f"trace kernel mean {sum(trace)/n:.1f} ms, fold_paths mean {(sum(times) - sum(trace))/n:.1f} ms",
                  flush=True)
    f.close()
    r.close()


if __name__ == "__main__":
    main()
