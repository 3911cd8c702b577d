"""Per-frame periods of a traced window loop (tools/prof_dropin256.sh): the
time between consecutive display copies, in ms, first N frames and summary.
usage: python tools/frame_periods.py DIR [N]"""
import csv
import glob
import statistics
import sys

root = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 24
cp = []
for p in glob.glob(root + "/**/*memory_copy_trace.csv", recursive=True):
    cp += [r for r in csv.DictReader(open(p)) if "DEVICE_TO_HOST" in r["Direction"]]
ends = sorted(int(r["End_Timestamp"]) for r in cp)
per = [(b - a) / 1e6 for a, b in zip(ends, ends[1:])][1:-1]  # from the last warm-up copy; no batch
print(" ".join(f"{x:.2f}" for x in per[:n]))
print(f"frames {len(per)} total {sum(per):.1f} ms median {statistics.median(per):.3f} "
      f"mean {statistics.mean(per):.3f} mean after {n}: {statistics.mean(per[n:]):.3f}")
