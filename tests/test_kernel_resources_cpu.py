"""Register budgets of the default-path kernels, read from the built library's
gfx950 code object (no GPU needed).

The hot kernels are HBM-bound and their rate follows occupancy: a change
that pushes an instantiation over a VGPR step (64 -> 8 waves per SIMD,
72 -> 7, 80 -> 6, 96 -> 5) costs it directly -- round 3 lost 10 % at 7-pt
256^3 to an unnoticed 75 -> 101 VGPR jump (profiles/r03_ab/vgpr_fix_ab.log).
This test pins each default instantiation's budget and forbids spills there.
"""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.path.join(ROOT, "hpccg-sycl_amd", "lib", "libhpccg_hip.so")
LLVM = "/opt/rocm/lib/llvm/bin"

# demangled-name fragment -> max VGPRs (the occupancy step each default runs at)
BUDGETS = {
    # 200^3 default: the ring pair kernel (LDS-bound at 2 blocks of 8 waves per CU)
    "k_spmv_a2r<true, 27, 3, false>": 80,
    # 100^3 default: direct kernel, fused p, 4 early slots, fused update (6 waves)
    "k_spmv_a<27, false, true, 4, false, true, false>": 80,
    "k_spmv_a<27, false, true, 4, true, true, false>": 80,
    # 7-pt 256^3 default: nt, fused p, 7 early slots, x triple, fused update (6 waves)
    "k_spmv_a<7, true, true, 7, true, true, false>": 80,
    # unfused direct kernel (several ranks over RCCL): 7 waves
    "k_spmv_a<27, false, true, 4, false, false, false>": 72,
    "k_spmv_a<7, true, true, 7, true, false, false>": 80,
    "k_update<false>": 64,
    # option resident_update: 4 waves per SIMD, so 1024 resident blocks hold
    # the 977 pair units of 100^3 at once (the host also checks occupancy)
    "k_spmv_ar<false, 3, 2>": 128,
    "k_spmv_ar<true, 3, 2>": 128,
    # the persistent CG launch (4 blocks per CU: every pair block of 100^3
    # resident); its multi-rank form (peer all-reduce + ghost pull) too
    "k_cg_persist<false, false, 3, 2, 3>": 128,
    "k_cg_persist<true, false, 3, 2, 3>": 128,
    "k_cg_persist<false, true, 3, 2, 3>": 128,
    "k_cg_persist<true, true, 3, 2, 3>": 128,
}


def _kernels():
    for tool in ("clang-offload-bundler", "llvm-readelf"):
        if not os.path.exists(os.path.join(LLVM, tool)):
            pytest.skip(f"{tool} not in {LLVM}")
    if not shutil.which("objcopy") or not shutil.which("c++filt"):
        pytest.skip("binutils missing")
    if not os.path.exists(LIB):
        pytest.skip("library not built (python -c 'import __graft_entry__ as g; g.build()')")
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        fb, co = os.path.join(d, "fb.bin"), os.path.join(d, "co.elf")
        subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fb}", LIB, os.path.join(d, "lib.copy")],
                       check=True, capture_output=True)
        subprocess.run([os.path.join(LLVM, "clang-offload-bundler"), "--unbundle", "--type=o", f"--input={fb}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True,
                       capture_output=True)
        notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True,
                               capture_output=True, text=True).stdout
    out, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s*\.(name|vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size):\s+(\S+)",
                     line)
        if not m:
            continue
        k, v = m.groups()
        if k == "name":
            cur = out.setdefault(v, {})
        elif cur is not None:
            cur[k] = int(v)
    names = list(out)
    dem = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout
    return {d.replace("hpccg::(anonymous namespace)::", ""): out[n] for n, d in zip(names, dem.splitlines())}


def test_default_kernels_within_register_budget():
    ks = _kernels()
    assert ks, "no kernels found in the gfx950 code object"
    for frag, budget in BUDGETS.items():
        hits = {n: r for n, r in ks.items() if frag in n}
        assert hits, f"{frag} not in the code object"
        for n, r in hits.items():
            assert r["vgpr_count"] <= budget, f"{n}: {r['vgpr_count']} VGPRs > budget {budget}"
            assert r.get("vgpr_spill_count", 0) == 0, f"{n}: VGPR spills"
            assert r.get("private_segment_fixed_size", 0) <= 32, f"{n}: scratch {r.get('private_segment_fixed_size')}"


def test_instantiation_count():
    """the variants that measured even or slower are out of
    the library -- one slot-loop shape each for the resident and persistent
    launches (the persistent one also in its multi-rank form), one LDS-DMA
    ring depth, the default prefetch depths (round 5's
    library held 140 kernels, round 4's 118)."""
    import collections
    ks = _kernels()
    by = collections.Counter(n.split("<")[0].split("(")[0].replace("void ", "") for n in ks)
    assert by["k_cg_persist"] == 4 and by["k_spmv_ar"] == 2, by  # (one- and multi-rank persistent forms)
    assert by["k_spmv_a2r"] <= 5, by  # (27, 7) x fused / not, + the timeline's
    assert "k_p_boundary" not in by
    assert len(ks) <= 80, len(ks)
