"""Summarise the rocprofv3 --pmc passes of tools/gpu_pmc.sh for one kernel.

usage: python tools/pmc_summary.py gpurun_out/<round>/pmc KERNEL_SUBSTR OUT.json [note] [samples_per_launch]

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and
WRITE_SIZE are in KiB; on gfx950 FETCH_SIZE counts 128-B read requests at
64 B, so it is doubled; WRITE_SIZE is taken as is. Infinity-Cache hits are
counted by both, so this is L2-miss (fabric) traffic, an upper bound on HBM.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kernel_durations(pmc_dir, kname):
    """Mean duration (s) of the kernel's dispatches in the passes' kernel traces."""
    d = []
    for f in sorted(glob.glob(os.path.join(pmc_dir, "*", "*kernel_trace.csv"))):
        for row in csv.DictReader(open(f)):
            if kname in row["Kernel_Name"]:
                d.append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return sum(d) / len(d) if d else None


def run_build(pmc_dir):
    """The code-object digest every profiled pass reported (its bench line's
    roofline.build, written to p<i>.out); the passes must agree."""
    builds = {}
    for f in sorted(glob.glob(os.path.join(pmc_dir, "p*.out"))):
        lines = [json.loads(x) for x in open(f) if x.startswith("{")]
        if not lines or not (lines[-1].get("roofline") or {}).get("build"):
            raise SystemExit(f"{f}: no bench line with roofline.build")
        builds[os.path.basename(f)] = lines[-1]["roofline"]["build"]
    if not builds:
        raise SystemExit(f"no p*.out bench lines under {pmc_dir}")
    if len(set(builds.values())) != 1:
        raise SystemExit(f"PMC passes ran different builds: {builds}")
    return next(iter(builds.values()))


# The scalar unit's issue ceiling, measured by tools/salu_peak.hip on the GPU box
# (profiles/r05/salu_peak.json): independent scalar ALU instructions per CU-cycle
# with every wave slot of the render kernels occupied.
SALU_PEAK_PER_CU_CYCLE = 1.0


def issue_fields(avg, cus=256):
    """Per-CU-cycle issue rates of the kernel from per-dispatch counters:
    scalar ALU (SQ_INSTS_SALU), branch (SQ_INSTS_BRANCH) and wave64 VALU
    instructions over 256 CUs x the kernel's cycles (GRBM_GUI_ACTIVE / 8 XCDs),
    the scalar rate against the measured scalar-unit ceiling, and the mean
    resident waves per CU (SQ_WAVE_CYCLES counts quad-cycles: x4) against the
    32 wave slots of a CU."""
    if "GRBM_GUI_ACTIVE" not in avg:
        return {}
    cu_cycles = cus * avg["GRBM_GUI_ACTIVE"] / 8
    out = {}
    if "SQ_INSTS_SALU" in avg:
        out["salu_per_cu_cycle"] = round(avg["SQ_INSTS_SALU"] / cu_cycles, 4)
        if SALU_PEAK_PER_CU_CYCLE:
            out["salu_issue_frac"] = round(out["salu_per_cu_cycle"] / SALU_PEAK_PER_CU_CYCLE, 4)
            out["salu_peak_per_cu_cycle"] = SALU_PEAK_PER_CU_CYCLE
    if "SQ_INSTS_BRANCH" in avg:
        out["branch_per_cu_cycle"] = round(avg["SQ_INSTS_BRANCH"] / cu_cycles, 4)
    if "SQ_INSTS_VALU" in avg:
        out["valu_per_cu_cycle"] = round(avg["SQ_INSTS_VALU"] / cu_cycles, 4)
    if "SQ_WAVE_CYCLES" in avg:
        waves = 4 * avg["SQ_WAVE_CYCLES"] / cu_cycles
        out["mean_waves_per_cu"] = round(waves, 2)
        out["occupancy_pct"] = round(100 * waves / 32, 2)
    return out


def main():
    pmc_dir, kname, out = sys.argv[1], sys.argv[2], sys.argv[3]
    note = sys.argv[4] if len(sys.argv) > 4 else ""
    samples = int(sys.argv[5]) if len(sys.argv) > 5 else 0  # samples one launch of the kernel renders
    vals = defaultdict(lambda: defaultdict(float))  # counter -> dispatch -> value
    meta = {}
    for f in sorted(glob.glob(os.path.join(pmc_dir, "*", "*counter_collection.csv"))):
        for row in csv.DictReader(open(f)):
            if kname not in row["Kernel_Name"]:
                continue
            key = (f, row["Dispatch_Id"])
            vals[row["Counter_Name"]][key] += float(row["Counter_Value"])
            meta = {"kernel": row["Kernel_Name"].split("(")[0], "vgpr": int(row["VGPR_Count"]),
                    "agpr": int(row["Accum_VGPR_Count"]), "sgpr": int(row["SGPR_Count"]),
                    "scratch_bytes_per_lane": int(row["Scratch_Size"]), "grid": int(row["Grid_Size"])}
    if not vals:
        raise SystemExit(f"no dispatches of {kname!r} under {pmc_dir}")
    avg = {c: sum(d.values()) / len(d) for c, d in vals.items()}
    res = dict(meta)
    # the build the counters belong to: bench.py replays this summary only onto
    # a run of the same code object (bench.build_id). Taken from the profiled
    # runs' own bench lines (roofline.build), not from the library on disk now,
    # so a summary of old counters is never stamped with a later build.
    res["code_object_sha256"] = run_build(pmc_dir)
    res["dispatches"] = {c: len(d) for c, d in vals.items()}
    res["counters_avg_per_dispatch"] = {c: round(v, 3) for c, v in sorted(avg.items())}
    if "FETCH_SIZE" in avg and "WRITE_SIZE" in avg:
        fetch = avg["FETCH_SIZE"] * 1024 * 2
        write = avg["WRITE_SIZE"] * 1024
        res["fetch_bytes_per_launch"] = fetch
        res["write_bytes_per_launch"] = write
        res["hbm_bytes_per_launch"] = round(fetch + write)
        if samples:
            res["samples_per_launch"] = samples
            res["hbm_bytes_per_sample"] = round((fetch + write) / samples, 2)
    if "TCC_HIT_sum" in avg and "TCC_MISS_sum" in avg:
        res["l2_hit_rate"] = round(avg["TCC_HIT_sum"] / max(avg["TCC_HIT_sum"] + avg["TCC_MISS_sum"], 1), 4)
    if "SQ_WAIT_ANY" in avg and "SQ_WAVE_CYCLES" in avg:
        res["wait_any_frac"] = round(avg["SQ_WAIT_ANY"] / max(avg["SQ_WAVE_CYCLES"], 1), 4)
    if "SQ_THREAD_CYCLES_VALU" in avg and "SQ_ACTIVE_INST_VALU" in avg:
        res["valu_lane_util"] = round(avg["SQ_THREAD_CYCLES_VALU"] / max(64 * avg["SQ_ACTIVE_INST_VALU"], 1), 4)
    if samples and "SQ_INSTS_VALU" in avg:
        res["valu_insts_per_sample"] = round(avg["SQ_INSTS_VALU"] / samples, 3)
        if "SQ_INSTS_SALU" in avg:
            res["salu_insts_per_sample"] = round(avg["SQ_INSTS_SALU"] / samples, 3)
    if samples and "SQ_ACTIVE_INST_VALU" in avg:
        # quad-cycles (4 SIMD cycles) of VALU issue per sample, summed over waves
        res["valu_active_quads_per_sample"] = round(avg["SQ_ACTIVE_INST_VALU"] / samples, 3)
    dur = kernel_durations(pmc_dir, kname)
    if dur:
        res["kernel_ms"] = round(dur * 1e3, 3)
    if "GRBM_GUI_ACTIVE" in avg and dur:
        # MI355X_MICROARCH.md (DVFS): effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time
        clock = avg["GRBM_GUI_ACTIVE"] / 8 / dur
        res["clock_ghz"] = round(clock / 1e9, 3)
        if "SQ_ACTIVE_INST_VALU" in avg:
            # VALUBusy (rocprof's gfx9 formula): VALU issue quad-cycles x 4 over the 1024 SIMDs' cycles.
            # On gfx950 it can exceed 1: two waves' wave64 FP32 instructions share a 4-cycle window
            res["valu_busy"] = round(avg["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * avg["GRBM_GUI_ACTIVE"] / 8), 4)
        if "SQ_INSTS_VALU" in avg:
            # VALU issue against its peak: a wave64 FP32 instruction every 2 cycles per SIMD
            # (MI355X_MICROARCH.md: v_fma_f32 wave64 2 cyc; = 157.3 TF FP32 at full lanes)
            res["valu_issue_frac"] = round(avg["SQ_INSTS_VALU"] * 2 / (1024 * avg["GRBM_GUI_ACTIVE"] / 8), 4)
    res.update(issue_fields(avg))
    res["method"] = ("rocprofv3 --pmc, one counter group per pass (tools/gpu_pmc.sh); FETCH_SIZE KiB x1024 x2 "
                     "(gfx950 half-count, MI355X_MICROARCH.md §HBM) + WRITE_SIZE KiB x1024; per dispatch average")
    if note:
        res["note"] = note
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
