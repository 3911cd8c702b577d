"""Register and scratch use of the kernels in libfsgpu.so, read from the
gfx950 code object's metadata (no GPU needed): the regression guard of
tests/test_isa_guard.py and a quick look for A/B builds.

usage: python tools/isa_guard.py [path/to/libfsgpu.so]
"""
import os
import re
import struct
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"
FIELDS = ("private_segment_fixed_size", "sgpr_count", "sgpr_spill_count", "vgpr_count", "vgpr_spill_count",
          "agpr_count", "group_segment_fixed_size")


def code_object(so_path, target="gfx950"):
    """The `target` code object of the clang offload bundle in a HIP shared library."""
    data = open(so_path, "rb").read()
    i = data.find(b"__CLANG_OFFLOAD_BUNDLE__")
    if i < 0:
        raise ValueError(f"{so_path}: no offload bundle")
    n = struct.unpack_from("<Q", data, i + 24)[0]
    p = i + 32
    for _ in range(n):
        off, size, tl = struct.unpack_from("<QQQ", data, p)
        p += 24
        triple = data[p:p + tl].decode()
        p += tl
        if triple.endswith(target) and size:
            return data[i + off:i + off + size]
    raise ValueError(f"{so_path}: no {target} code object")


def demangle_lean(name):
    """render_kernel_lean<b, W, b, ...> as fs_last_kernel names it."""
    m = re.search(r"render_kernel_leanIL(b[01])ELi(\d+)E((?:L(?:b[01])E)+)", name)
    if not m:
        return None
    b = lambda t: "true" if t == "b1" else "false"  # noqa: E731
    rest = [b(t) for t in re.findall(r"L(b[01])E", m.group(3))]
    return f"render_kernel_lean<{b(m.group(1))}, {m.group(2)}, " + ", ".join(rest) + ">"


def kernel_resources(so_path=None):
    so_path = so_path or os.path.join(ROOT, "final-stage-path-tracer-2-0_amd", "libfsgpu.so")
    with tempfile.NamedTemporaryFile(suffix=".co") as f:
        f.write(code_object(so_path))
        f.flush()
        out = subprocess.run([READELF, "--notes", f.name], check=True, capture_output=True, text=True).stdout
    # amdhsa.kernels: one YAML list item per kernel ("  - .agpr_count: ..."),
    # keys in alphabetical order (.name comes after some of the counts);
    # the nested .args items are deeper and name no FIELDS
    res, cur, name = {}, None, None
    in_kernels = False
    for raw in out.splitlines():
        line = raw.strip()
        if line.startswith("amdhsa.kernels:"):
            in_kernels = True
            continue
        if not in_kernels:
            continue
        indent = len(raw) - len(raw.lstrip())
        if line.startswith("- .") and indent <= 2:
            if cur is not None and name:
                res[name] = cur
            cur, name = {}, None
            line = line[2:]
        if cur is None or not line.startswith("."):
            continue
        k, _, v = line[1:].partition(":")
        if k == "name" and indent <= 4:
            name = v.strip()
        elif k in FIELDS:
            cur[k] = int(v.strip())
    if cur is not None and name:
        res[name] = cur
    return res


if __name__ == "__main__":
    for name, r in kernel_resources(sys.argv[1] if len(sys.argv) > 1 else None).items():
        short = demangle_lean(name) or name.split("ENS_")[0]
        print(f"{short:60s} " + " ".join(f"{k}={r.get(k)}" for k in FIELDS))
