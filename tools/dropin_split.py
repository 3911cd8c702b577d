"""Per-frame time split of the drop-in window loop (examples/dropin_rate under
rocprofv3 --kernel-trace --memory-copy-trace): for each displayed frame the
trace kernel, fold_paths, fills, the display copy and the gaps between them
(host round trips), medians over the loop's frames (measurement aid, DESIGN
§6). usage: python tools/dropin_split.py PROFILE_DIR"""
import csv
import glob
import os
import statistics
import sys


def rows(pattern, root):
    out = []
    for p in glob.glob(os.path.join(root, "**", pattern), recursive=True):
        with open(p) as f:
            out += list(csv.DictReader(f))
    return out


def classify(name):
    if name.startswith("render_kernel") or "render_kernel_lean" in name:
        return "trace"
    if "fold_paths" in name:
        return "fold"
    if "fill" in name.lower() or "memset" in name.lower():
        return "fill"
    return "other"


def main(root):
    ev = []
    for r in rows("*kernel_trace.csv", root):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), classify(r["Kernel_Name"]), r["Kernel_Name"]))
    for r in rows("*memory_copy_trace.csv", root):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "copy_" + r.get("Direction", "?"), "copy"))
    ev.sort()
    # frames: each starts at a trace-kernel launch of one 1-spp frame; the last
    # trace launches belong to the batched submission and are dropped with it
    starts = [i for i, e in enumerate(ev) if e[2] == "trace"]
    if len(starts) < 8:
        raise SystemExit(f"only {len(starts)} trace launches in {root}")
    frames = []
    for a, b in zip(starts[1:-2], starts[2:-1]):  # skip the warm-up frame and the batch tail
        seg = ev[a:b]
        d = {}
        for s, e, k, _ in seg:
            d[k] = d.get(k, 0) + (e - s)
        d["period"] = ev[b][0] - ev[a][0]
        d["busy"] = sum(e - s for s, e, _, _ in seg)
        d["gaps"] = d["period"] - d["busy"]
        frames.append(d)
    keys = sorted({k for f in frames for k in f})
    print(f"# {len(frames)} frames from {root}; medians in us")
    for k in keys:
        vals = [f.get(k, 0) / 1e3 for f in frames]
        print(f"{k:>16}: {statistics.median(vals):9.1f}  (min {min(vals):.1f}, max {max(vals):.1f})")
    names = sorted({n for _, _, k, n in ev if k in ("trace", "fold")})
    print("kernels:", "; ".join(names))


if __name__ == "__main__":
    main(sys.argv[1])
