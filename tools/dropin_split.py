"""Per-frame timeline of the drop-in window loop (examples/dropin_rate under
rocprofv3 --kernel-trace --memory-copy-trace): for each displayed frame the
fold of its samples, the display copy to the host and the gaps between them,
and how the trace that made the samples lines up with its fold (with the
lookahead, fs_options.lookahead, traces run ahead of their folds on other
streams). Medians over the loop's frames, in us (measurement aid, DESIGN §6;
VERDICT r5 item 3). usage: python tools/dropin_split.py PROFILE_DIR"""
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


def main(root):
    traces, folds, copies = [], [], []
    for r in rows("*kernel_trace.csv", root):
        ev = (int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
        if "render_kernel_lean" in r["Kernel_Name"]:
            traces.append(ev)
        elif "fold_paths" in r["Kernel_Name"]:
            folds.append(ev)
    for r in rows("*memory_copy_trace.csv", root):
        if "DEVICE_TO_HOST" in r.get("Direction", ""):
            copies.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    traces.sort()
    folds.sort()
    copies.sort()
    if len(folds) < 8:
        raise SystemExit(f"only {len(folds)} folds in {root}")
    # frame k: fold k and the first display copy after it; the k-th trace made
    # its samples (traces start in sample order). Skip the two warm-up frames
    # (dropin_rate's untimed calls) and the batched submission at the end (its
    # fold has no copy before the last).
    frames = []
    ci = 0
    for k in range(2, len(folds) - 2):
        fs, fe = folds[k]
        while ci < len(copies) and copies[ci][0] < fe:
            ci += 1
        if ci >= len(copies):
            break
        cs, ce = copies[ci]
        nxt = folds[k + 1][0]
        d = {"period": nxt - fs, "fold": fe - fs, "fold_to_copy": cs - fe, "copy": ce - cs,
             "copy_to_next_fold": nxt - ce}
        if k < len(traces):
            ts, te = traces[k]
            d["trace"] = te - ts
            d["trace_end_to_fold_start"] = fs - te  # > 0: the fold did not wait for its trace
        frames.append(d)
    print(f"# {len(frames)} frames from {root}; medians in us (min, max)")
    for key in ("period", "fold", "fold_to_copy", "copy", "copy_to_next_fold", "trace", "trace_end_to_fold_start"):
        vals = [f[key] / 1e3 for f in frames if key in f]
        if vals:
            print(f"{key:>24}: {statistics.median(vals):9.1f}  ({min(vals):.1f}, {max(vals):.1f})")
    print(f"traces {len(traces)}, folds {len(folds)}, display copies {len(copies)}")


if __name__ == "__main__":
    main(sys.argv[1])
