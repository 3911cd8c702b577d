"""ISA regression guard (CPU): the product trace kernels' scratch, register
spills and VGPR budget, read from the gfx950 code object in libfsgpu.so.

Several of the kernel's measured gains rest on how the compiler allocates
registers (DESIGN_HISTORY.md §5: cold records read at their use, the integer-min
slab clamp, the 6-wave launch bound); every 8-16 B/lane of extra spills has
cost 1-2 %. A toolchain update or a source change that undoes them fails
here before it reaches a GPU. Raising a limit is a deliberate edit, made
with the A/B that justifies it."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
import isa_guard  # noqa: E402

# kernel (as fs_last_kernel names it) -> (max scratch B/lane, max SGPR spills, VGPRs)
LIMITS = {
    # PARKED schedule: C3 and C4 (the bench kernel). 60 -> 40 B/lane once the
    # backward pass left the kernel for fold_paths (round 4: C4 +4.5 %,
    # profiles/r04/ab_records.log); 40 -> 28 without SLP vectorization (round 5:
    # C4 +7.4 %, profiles/r05/ab_noslp.log); 28 -> 48 with the node step as
    # selects (C4 +2.8 %, profiles/r05/ab_nodesel.log); 48 -> 20 once the
    # cuboid cull took the segment's slopes instead of three v_rcp of its own
    # that the compiler hoisted out of the object loop and spilled (C4 +4 %,
    # C2 +5 %, write-backs 176 -> 95 B per sample, profiles/r05/ab_spills.log)
    "render_kernel_lean<false, 6, false, true, false, false, false, false>": (24, 14, 80),
    # LEAN schedule: scenes with BVH walks and no large mesh (no bench config
    # runs it). 24 -> 12 B/lane with the cuboid cull on the segment's slopes,
    # 20 with the zero-length shortcut (its division behind a branch)
    "render_kernel_lean<false, 6, false, false, false, false, false, false>": (24, 14, 80),
    # LEAN without walks (NOWALK: every mesh small, no walk stack, 8 waves per
    # SIMD): C1 and C2. 44 -> 40 B/lane without the backward pass (C2 +8.5 %);
    # 40 -> 48 with the round-5 face loop and no SLP vectorization (C2 +8.9 %,
    # profiles/r05/ab_noslp.log); 48 -> 24 with the cuboid cull on the
    # segment's slopes (profiles/r05/ab_spills.log)
    "render_kernel_lean<false, 8, false, false, false, false, true, false>": (24, 16, 64),
    # The TRIG twins (round 6: a thin-lens camera or frosted glass; the host
    # libm's sinf/cosf restated in double, csrc/fs_libm.h): the parked-walk
    # kernel reserves 28 B/lane, its one spilled value reloaded only on Fog paths
    "render_kernel_lean<false, 6, false, true, false, false, false, true>": (28, 14, 80),
    "render_kernel_lean<false, 6, false, false, false, false, false, true>": (24, 14, 80),
    "render_kernel_lean<false, 8, false, false, false, false, true, true>": (24, 16, 64),
}


@pytest.fixture(scope="module")
def resources():
    if not os.path.exists(isa_guard.READELF):
        pytest.skip("llvm-readelf not in this image")
    return {isa_guard.demangle_lean(k): v for k, v in isa_guard.kernel_resources().items()
            if isa_guard.demangle_lean(k)}


@pytest.mark.parametrize("kernel", sorted(LIMITS))
def test_trace_kernel_spills_within_budget(kernel, resources):
    assert kernel in resources, f"{kernel} not in libfsgpu.so"
    r = resources[kernel]
    scratch, sgpr_spills, vgprs = LIMITS[kernel]
    assert r["private_segment_fixed_size"] <= scratch, r
    assert r["sgpr_spill_count"] <= sgpr_spills, r
    assert r["vgpr_count"] <= vgprs, r  # the kernel's waves per SIMD


def test_every_product_kernel_fits_its_wave_count(resources):
    """render_kernel_lean<COUNT, waves, ...>: the VGPRs and LDS of a product
    kernel fit `waves` waves per SIMD (512 VGPRs per lane and 160 KiB of LDS
    per CU of 4 SIMDs)."""
    for name, r in resources.items():
        if name.startswith("render_kernel_lean<false"):
            waves = int(name.split(", ")[1])
            assert r["vgpr_count"] <= 512 // waves // 8 * 8, (name, r)
            assert r["group_segment_fixed_size"] <= 160 * 1024 // (4 * waves), (name, r)


def test_lookahead_fold_fits_beside_background_waves():
    """fold_paths_lite (the fold of a lookahead call) without scratch, in at
    most 56 VGPRs on untextured scenes (64 textured): bg_waves leaves room for
    four of its waves per SIMD beside a background trace launch (C4 3 x 80 +
    4 x 56 <= 512, C2 4 x 64 + 4 x 56), so the window loop's folds never wait
    for a trace launch to drain."""
    if not os.path.exists(isa_guard.READELF):
        pytest.skip("llvm-readelf not in this image")
    lite = {k: v for k, v in isa_guard.kernel_resources().items() if "fold_paths_lite" in k}
    assert len(lite) == 8, sorted(lite)
    for name, r in lite.items():
        tex = name.startswith("_ZN2fs3dev15fold_paths_liteILb1")
        assert r["vgpr_count"] <= (64 if tex else 56) and r["private_segment_fixed_size"] == 0, (name, r)
