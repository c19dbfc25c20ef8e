"""Code-generation guard for the shipped gfx950 kernels (CPU test, reads the built library).

hipcc's register allocation is fragile on these hand-scheduled kernels: a small source change once
made it re-derive a value inside a rare branch of the FastCDC scan (256 VGPRs, spills to scratch,
3x slower) while every parity test still passed. This test extracts the gfx950 code object from
oxen_amd/liboxen_hash.so and checks every kernel's metadata: no VGPR spills, no scratch.
"""
import os
import re
import shutil
import subprocess

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"


def _kernel_metadata(lib, tmp_path):
    fatbin = tmp_path / "fatbin.bin"
    subprocess.run(["objcopy", f"--dump-section=.hip_fatbin={fatbin}", lib, str(tmp_path / "lib_copy.so")], check=True)
    # the section holds one offload bundle per translation unit, back to back
    data = fatbin.read_bytes()
    magic = b"__CLANG_OFFLOAD_BUNDLE__"
    starts = [m.start() for m in re.finditer(re.escape(magic), data)] + [len(data)]
    notes = ""
    for b, (lo, hi) in enumerate(zip(starts, starts[1:])):
        part, co = tmp_path / f"bundle{b}.bin", tmp_path / f"co{b}.o"
        part.write_bytes(data[lo:hi])
        subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={part}",
                        "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
        notes += subprocess.run([f"{LLVM}/llvm-readelf", "--notes", str(co)], capture_output=True, text=True,
                                check=True).stdout
    kernels, cur = {}, None
    for line in notes.splitlines():
        m = re.match(r"\s+\.(name|vgpr_count|vgpr_spill_count|sgpr_spill_count|private_segment_fixed_size):\s+(\S+)", line)
        if not m:
            continue
        if m.group(1) == "name":
            cur = kernels.setdefault(m.group(2), {})
        elif cur is not None:
            cur[m.group(1)] = int(m.group(2))
    return kernels


@pytest.mark.skipif(not os.path.exists(f"{LLVM}/clang-offload-bundler") or not shutil.which("objcopy"),
                    reason="ROCm LLVM tools not present")
def test_kernels_do_not_spill(built_lib, tmp_path):
    from oxen_amd import build

    k = _kernel_metadata(build.LIB, tmp_path)
    assert any("cdc_scan_kernel" in n for n in k) and any("xxh3_wave_kernel" in n for n in k), sorted(k)
    # SGPR spills go to VGPR lanes (no memory traffic) and are tolerated; VGPR spills and scratch are not
    bad = {n: v for n, v in k.items() if v.get("vgpr_spill_count", 0) or v.get("private_segment_fixed_size", 0)}
    assert not bad, bad
    # the lane-major scan runs 12 waves per workgroup (3 per SIMD): at most 168 VGPRs (512 / 3, in
    # granules of 8), or the workgroup cannot launch
    scan = [v for n, v in k.items() if "cdc_scan_kernel" in n]
    assert all(v["vgpr_count"] <= 168 for v in scan), scan
