#!/bin/bash
# Keyswitch at latency-level batch sizes: split contraction (default build) vs build_variants/$1,
# after the PBS and radix parity tests.  Output: gpurun_out/kss_$1.txt
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_pbs_gpu.py tests/test_radix_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/kss_t.log 2>&1 || exit 1
for B in 64 256 1024 8192; do
  timeout -k 10 120 python tools/pbs_probe.py $B 6 >> gpurun_out/kss_$1.txt 2>&1 || exit 2
  FHE_PROBE_PKG=build_variants/$1 timeout -k 10 120 python tools/pbs_probe.py $B 6 >> gpurun_out/kss_$1.txt 2>&1 || exit 3
done
