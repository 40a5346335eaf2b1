#!/bin/bash
# round 4: latency-kernel A/B (br_wx vs br_wide) + throughput A/B (qx layout fix), then the PBS tests
set -o pipefail
OUT=gpurun_out/${1:-r4e}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/lat_ab.py 5 > $OUT/lat_ab.txt 2>&1 || { tail -20 $OUT/lat_ab.txt; exit 1; }
cat $OUT/lat_ab.txt
timeout -k 10 300 python3 -u tools/br_ab.py 32768 4 > $OUT/br_ab.txt 2>&1 || { tail -20 $OUT/br_ab.txt; exit 2; }
cat $OUT/br_ab.txt
timeout -k 10 900 python3 -u -m pytest tests/test_pbs_gpu.py -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 3; }
tail -3 $OUT/gpu_tests.txt
