"""Occupancy guard for the blind-rotate and keyswitch kernels (CPU: compiles device code, reads the code-object
descriptors).  Each kernel is designed for a fixed occupancy: a register total
(arch VGPR + AGPR) above 256 silently halves occupancy -- it happened once through a VGPR->AGPR
spill (next_free_vgpr 258) and cost 50% of throughput -- and scratch spills in the CMUX loop
stall it.  Both are checked here so such a change fails a test instead of a benchmark."""
import os
import re
import shutil
import subprocess

import pytest

from conftest import ROOT

CSRC = os.path.join(ROOT, "fhe-sign_amd", "csrc")
HIPCC = "/opt/rocm/bin/hipcc"


def descriptors(src, tmp_path, flags=()):
    out = tmp_path / (os.path.basename(src) + ".s")
    subprocess.run([HIPCC, "-O3", "-std=c++17", "-ffp-contract=off", "--offload-arch=gfx950", "--cuda-device-only",
                    "-S", *flags, "-I", os.path.join(ROOT, "include"), "-I", CSRC, src, "-o", str(out)],
                   check=True, capture_output=True)
    s = out.read_text()
    res = {}
    for m in re.finditer(r"\.amdhsa_kernel (\S+)\n(.*?)\.end_amdhsa_kernel", s, re.S):
        f = dict(re.findall(r"\.amdhsa_(\w+) (\d+)", m.group(2)))
        res[m.group(1)] = {k: int(v) for k, v in f.items()}
    return res


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,flags,kernel,lds_per_cu_ok,max_regs,max_scratch", [
    ("br_wide.hip", (), "k_blind_rotate_wideILi1", 1, 256, 0),  # one 8-wave workgroup per CU (classic)
    ("br_wide.hip", (), "k_blind_rotate_wideILi2", 1, 256, 0),  # the same, multi-bit
    ("br_qy.hip", ("-mllvm", "-amdgpu-sched-strategy=max-memory-clause"), "k_blind_rotate_qyILi1", 3, 168, 0),  # classic: 3 four-wave workgroups per CU, 3 waves/SIMD
    ("br_qy.hip", ("-mllvm", "-amdgpu-sched-strategy=max-memory-clause"), "k_blind_rotate_qyILi2", 2, 256, 0),  # multi-bit: 2 per CU, 2 waves/SIMD
    ("br_qy.hip", ("-mllvm", "-amdgpu-sched-strategy=max-memory-clause"), "k_blind_rotate_qy2ILi1", 2, 256, 0),  # classic, two ciphertexts per workgroup: 2 per CU
    ("br_qy.hip", ("-mllvm", "-amdgpu-sched-strategy=max-memory-clause"), "k_blind_rotate_qy2ILi2", 1, 256, 0),  # 8-wave variant: 1 per CU
    ("ks_mfma.hip", (), "k_ks_mfmaILi2", 3, 168, 0),  # keyswitch, latency levels: 3 workgroups per CU
    ("ks_mfma.hip", (), "k_ks_mfmaILi4", 2, 512, 0),  # keyswitch, large batches: one wave per SIMD, no spill
])
def test_blind_rotate_occupancy(tmp_path, src, flags, kernel, lds_per_cu_ok, max_regs, max_scratch):
    d = descriptors(os.path.join(CSRC, src), tmp_path, flags)
    ks = [v for k, v in d.items() if kernel in k]
    assert ks, f"{kernel} not found in {src}"
    for f in ks:
        total = max(f["next_free_vgpr"], f["accum_offset"])
        assert total <= max_regs, f"{kernel}: {f['next_free_vgpr']} registers -> below the designed occupancy"
        assert f["private_segment_fixed_size"] <= max_scratch, f"{kernel}: scratch spill"
        assert f["group_segment_fixed_size"] * lds_per_cu_ok <= 160 * 1024, f"{kernel}: LDS limits occupancy"
