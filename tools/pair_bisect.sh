#!/bin/bash
# Pair-kernel timing (FHE_BR_KERNEL=2) of the default build and of build_variants/$@ at B = 8192 and
# 32768, the default build's quad kernel beside them, after the pair parity tests.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py -x -q --timeout 200 --timeout-method thread -k "pair or wide_and_quad" > gpurun_out/pair_t.log 2>&1 || exit 1
for B in 8192 32768; do
  echo "quad" >> gpurun_out/pair_bisect.txt
  timeout -k 10 150 python tools/variant_probe.py fhe-sign_amd $B 3 >> gpurun_out/pair_bisect.txt 2>&1 || exit 2
  for v in fhe-sign_amd "$@"; do
    [ "$v" = fhe-sign_amd ] || v=build_variants/$v
    echo "pair $v" >> gpurun_out/pair_bisect.txt
    FHE_BR_KERNEL=2 timeout -k 10 150 python tools/variant_probe.py $v $B 3 >> gpurun_out/pair_bisect.txt 2>&1 || exit 3
  done
done
