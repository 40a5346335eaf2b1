#!/bin/bash
# Same-box A/B of the multi-bit throughput kernel: default build vs build_variants/$1 at 32768,
# two repetitions, after the PBS parity tests.  Output: gpurun_out/mb_ab_$1.txt
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/mb_t.log 2>&1 || exit 1
export FHE_PROBE_MB=1
for rep in 1 2; do
  for v in fhe-sign_amd build_variants/$1; do
    timeout -k 10 150 python tools/variant_probe.py $v 32768 3 >> gpurun_out/mb_ab_$1.txt 2>&1 || exit 2
  done
done
