#!/bin/bash
# Same-box A/B of the 4-wave kernel's MAC: split around the digit-swap barrier (default build) vs
# the 4-deep BSK ring (build_variants/q_nosplit), plus the PBS parity tests.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/qs_t.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 120 python tools/variant_probe.py fhe-sign_amd 8192 4 >> gpurun_out/qs_ab.txt 2>&1 || exit 2
  timeout -k 10 120 python tools/variant_probe.py build_variants/q_nosplit 8192 4 >> gpurun_out/qs_ab.txt 2>&1 || exit 3
done
