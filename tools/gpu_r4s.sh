#!/bin/bash
# qy with early key loads (default): blind-rotate parity tests, then untwist-load placement variants
set -o pipefail
OUT=gpurun_out/${1:-r4s}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_pbs_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
bash tools/gpu_sched_ab.sh ${1:-r4s}/sab 3
