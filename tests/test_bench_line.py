"""bench.py's stdout line (CPU, no GPU): the driver keeps only the last 8 KB of stdout, and round 5's
14.4 KB line lost the default-parameter mul / sign seconds to that cut.  compose_line is fed the full set
of legs bench.py runs (leg names read from bench.py itself) with realistic values; the line must stay under
LINE_MAX_BYTES with the classic headline keys in its last 2 KB, and everything else in the detail file."""
import argparse
import json
import os
import re
import sys

import pytest

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

LEGS = re.findall(r'leg\("(\w+)"', open(os.path.join(ROOT, "bench.py")).read())


def _ops(scale):
    ops = {name: {"seconds": 0.0123456789 * scale * (i + 1), "runs": [0.0123456789 * scale] * bench.OPS_REPS,
                  "pbs": 57564 + i, "levels": 44 + i} for i, name in enumerate(LEGS)}
    ops["sign_fhe_with_k0_batch8_compat"]["signs_per_s"] = 2.93456789
    return ops


def _pbs_part(kind):
    lat = {"before_throughput": {"B=1": 1.987654321, "B=256": 2.3987654321},
           "after_throughput": {"B=1": 1.998765432, "B=256": 2.4187654321}}
    hbm = {"bound": "hbm", "achieved": 3456.789012, "peak": 8000.0, "unit": "GB/s", "frac": 0.43209876}
    l2 = dict(hbm, bound="l2_to_cu", bytes_per_launch=1791500000000, peak=34500.0)
    roof = {"bound": "fp64_valu", "compute_pipe": "fp64 VALU (FFT butterflies; no dense contraction on the path)",
            "kernel": f"k_blind_rotate_qy<{1 if kind == 'classic' else 2}>", "achieved": 31.23456789, "peak": 78.6,
            "unit": "TFLOP/s", "frac": 0.397654321, "peak_measured": 65.0, "frac_measured": 0.48123456789,
            "flops_per_pbs": 218628096, "kernel_ms": 229.87654321, "keyswitch_ms": 2.987654321, "hbm": hbm, "l2": l2}
    return {"value": 138582.123456, "ms_per_step": 236.4567891234,
            "params": "n=834,N=2048,k=1,pbs=2^23x1,ks=2^3x5,msg=4,carry=4,grouping=1", "roofline": roof,
            "pcie_inclusive_pbs_per_s": 101234.56789, "latency_level_ms": lat,
            "clock": {"shader_ghz": 2.0312345678, "cu_cycles_per_pbs": 3754123.456789, "br_cu_cycles_per_pbs": 3654123.4,
                      "wg_cycles": 11234567.891, "workgroups": 655360, "source": "s_memtime / s_memrealtime ..."}}


def _cpu():
    ops = {n: {"seconds": 123.456789, "how": "projected", "pbs": 57564, "levels": 44, "projected_seconds": 120.1}
           for n in bench.CPU_REPLAY_OPS + bench.CPU_PROJECT_OPS}
    return {"value": 1236.123456, "unit": "PBS/s", "cores": 16, "kind": "port", "nproc": 256, "affinity": 16,
            "cgroup_cpu_quota": 16.0, "simd": "avx512",
            "sample": "19744 PBS (KS+BR+SE, same params/keys shape) with the C oracle (bit-exact restatement; its "
                      "blind rotation and keyswitch loops in AVX2 / AVX-512 ...), OpenMP 16 threads = ..., 12.3 s",
            "ops": ops, "ops_note": "x" * 400}


@pytest.mark.parametrize("world", [1, 8])
def test_line_short_with_headline_last(tmp_path, world):
    a = bench.parse(["--detail", str(tmp_path / "detail.json")])
    mb = dict(_pbs_part("multibit"), ops=_ops(0.8))
    fan = None
    if world > 1:
        fan = {"ranks": world, "min_level": 257}
        for n in ("warmup_add_fast", "biguint256_mul_fast", "biguint256_mul_compat", "sign_fhe_with_k0_v0_compat",
                  "sign_fhe_with_k0_v0_fast"):
            fan[n] = {"seconds": 0.1234567, "ok": True, "split_levels": 32}
    line, detail = bench.compose_line(a, world, _pbs_part("classic"), _ops(1.0), mb, fan,
                                      _cpu() if world == 1 else None)
    text = json.dumps(line, separators=(",", ":"))
    assert len(text.encode()) < bench.LINE_MAX_BYTES, len(text)
    tail = text[-2048:]
    for key in bench.HEADLINE_KEYS:
        assert f'"{key}":' in tail, key
    assert list(line)[-len(bench.HEADLINE_KEYS):] == list(bench.HEADLINE_KEYS)
    # the contract keys and the two required objects
    for key in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
                "vs_baseline", "dtype", "data", "config", "roofline"):
        assert key in line
    for key in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert key in line["roofline"]
    assert line["clock"]["shader_ghz"] > 0 and line["clock"]["cu_cycles_per_pbs"] > 0
    if world == 1:
        for key in ("value", "unit", "cores", "kind", "sample"):
            assert key in line["cpu_baseline"]
    # everything dropped from the line is in the detail file
    assert detail["ops"]["biguint256_mul_compat"]["runs"]
    assert "multibit_ops" in detail and "vs_reference_readme" in detail
    assert "sign_fhe_with_k0_v0_callsite" in LEGS and "sign_fhe_with_k0_v0_callsite" in line["ops_s"]
    json.dumps(detail)
