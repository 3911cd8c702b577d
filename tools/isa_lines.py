"""Static instruction counts of one render kernel per source line range, from a
debug-info device build (no GPU needed): which source regions the compiler
turned into how many VALU / SALU / memory instructions.

usage: python tools/isa_lines.py KERNEL_PREFIX [file:first-last ...]
  KERNEL_PREFIX  template arguments of render_kernel_lean as in its mangled
                 name, e.g. Lb0ELi8ELb0ELb0ELb0ELb0ELb1ELb0E (NOWALK)
  ranges         e.g. fs_device.hip:208-256 (default: a per-line top list)

Builds csrc/fs_device.hip with -g for gfx950 into /tmp (a minute), then
disassembles with llvm-objdump --line-numbers. Instructions are attributed to
the innermost source line the line table gives them (inlined code counts at
the line of the inlined function's body).
"""
import collections
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_guard  # noqa: E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "final-stage-path-tracer-2-0_amd")
OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def build(out="/tmp/fs_isa_lines.o", extra=()):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-g", "-std=c++17", "-ffp-contract=off",
           "-fno-slp-vectorize", "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"), "--cuda-device-only", "-c",
           os.path.join(PKG, "csrc", "fs_device.hip"), "-o", out, *extra]
    subprocess.run(cmd, check=True)
    co = out + ".co"
    with open(co, "wb") as f:
        f.write(isa_guard.code_object(out))
    return co


def kind(mnem):
    if mnem.startswith("v_"):
        return "valu"
    if mnem.startswith(("s_load", "s_buffer_load")):
        return "smem"
    if mnem.startswith(("global_", "buffer_", "flat_", "scratch_")):
        return "vmem"
    if mnem.startswith("ds_"):
        return "lds"
    if mnem.startswith("s_"):
        return "salu"
    return "other"


def attribute(co, prefix):
    syms = subprocess.run([OBJDUMP, "-t", co], check=True, capture_output=True, text=True).stdout
    name = None
    for line in syms.splitlines():
        f = line.split()
        if f and "render_kernel_lean" + "I" + prefix in f[-1] and not re.search(r"\.(kd|[a-z_]+)$", f[-1]):
            name = f[-1]
    if not name:
        raise SystemExit(f"no kernel with template arguments {prefix}")
    dis = subprocess.run([OBJDUMP, "-d", "-l", "--no-show-raw-insn", f"--disassemble-symbols={name}", co],
                         check=True, capture_output=True, text=True).stdout
    cur = ("?", 0)
    rows = []
    for line in dis.splitlines():
        m = re.match(r"^; (/\S+):(\d+)", line)
        if m:
            cur = (os.path.basename(m.group(1)), int(m.group(2)))
            continue
        m = re.match(r"^\s+([sv]_\w+|global_\w+|buffer_\w+|flat_\w+|scratch_\w+|ds_\w+)", line)
        if m:
            rows.append((cur, m.group(1)))
    return name, rows


def main():
    prefix = sys.argv[1] if len(sys.argv) > 1 else "Lb0ELi6ELb0ELb1ELb0ELb0ELb0ELb0E"
    ranges = [a for a in sys.argv[2:] if a != "--scratch"]
    co = build()
    name, rows = attribute(co, prefix)
    total = collections.Counter(kind(m) for _, m in rows)
    print(f"{name[:90]}...: {len(rows)} instructions {dict(total)}")
    if "--scratch" in sys.argv:
        # where the spills are: scratch loads and stores by source line
        sc = collections.Counter((f, ln, m) for (f, ln), m in rows if m.startswith("scratch_"))
        for (f, ln, m), n in sorted(sc.items(), key=lambda kv: (kv[0][0], kv[0][1])):
            print(f"{f}:{ln}  {m} x{n}")
        return
    if ranges:
        for rg in ranges:
            fname, span = rg.split(":")
            a, b = (int(x) for x in span.split("-"))
            c = collections.Counter(kind(m) for (f, ln), m in rows if f == fname and a <= ln <= b)
            print(f"{rg}: {sum(c.values())} {dict(c)}")
    else:
        per = collections.Counter()
        for (f, ln), m in rows:
            if kind(m) == "valu":
                per[(f, ln)] += 1
        for (f, ln), n in per.most_common(40):
            print(f"{f}:{ln}  {n} valu")


if __name__ == "__main__":
    main()
