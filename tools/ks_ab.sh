#!/bin/bash
# Keyswitch A/B: PBS tests (incl. both keyswitch kernels at 4160), then the KS time of the default
# build vs build_variants/$1 at 8192 and 32768 (variant_probe prints BR; ks times from pbs_probe).
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/ks_t.log 2>&1 || exit 1
for B in 8192 32768; do
  timeout -k 10 120 python tools/pbs_probe.py $B 4 >> gpurun_out/ks_ab.txt 2>&1 || exit 2
  FHE_PROBE_PKG=build_variants/$1 timeout -k 10 120 python tools/pbs_probe.py $B 4 >> gpurun_out/ks_ab.txt 2>&1 || exit 3
done
