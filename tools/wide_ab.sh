#!/bin/bash
# Same-box A/B of the latency kernel (default build vs build_variants/$1) at B = 1, 128, 256, classic
# and multi-bit (both template instances: a change can help one and hurt the other), after the PBS
# parity tests.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/w_t.log 2>&1 || exit 1
for rep in 1 2; do
  for mb in 0 1; do
    for B in 1 128 256; do
      for v in fhe-sign_amd build_variants/$1; do
        FHE_PROBE_MB=$mb timeout -k 10 60 python tools/variant_probe.py $v $B 6 distinct >> gpurun_out/w_ab.txt 2>&1 || exit 2
      done
    done
  done
done
