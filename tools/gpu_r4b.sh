#!/bin/bash
# round 4: throughput-kernel A/B (br_qx vs br_quad, same box) then the PBS, 256-bit and fan-out GPU tests
set -o pipefail
OUT=gpurun_out/${1:-r4b}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/br_ab.py 32768 4 > $OUT/br_ab.txt 2>&1 || { cat $OUT/br_ab.txt | tail -20; exit 1; }
cat $OUT/br_ab.txt
timeout -k 10 900 python3 -u -m pytest tests/test_pbs_gpu.py tests/test_radix256_gpu.py tests/test_fanout_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 2; }
tail -3 $OUT/gpu_tests.txt
