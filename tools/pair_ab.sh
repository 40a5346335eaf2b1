#!/bin/bash
# Pair-kernel check on the GPU box: its parity tests, then a same-box A/B of the throughput kernels
# (br_pair.hip vs br_quad.hip) at B = 8192 and 32768.  Output under gpurun_out/.
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py -x -v --timeout 200 --timeout-method thread -k "pair or wide_and_quad" > gpurun_out/pair_t.log 2>&1 || exit 1
echo "pair:" > gpurun_out/pair_ab.txt
FHE_BR_KERNEL=2 timeout -k 10 120 python tools/variant_probe.py fhe-sign_amd 8192 4 >> gpurun_out/pair_ab.txt 2>&1 || exit 2
echo "quad:" >> gpurun_out/pair_ab.txt
timeout -k 10 120 python tools/variant_probe.py fhe-sign_amd 8192 4 >> gpurun_out/pair_ab.txt 2>&1 || exit 3
echo "pair 32768:" >> gpurun_out/pair_ab.txt
FHE_BR_KERNEL=2 timeout -k 10 120 python tools/variant_probe.py fhe-sign_amd 32768 3 >> gpurun_out/pair_ab.txt 2>&1 || exit 4
