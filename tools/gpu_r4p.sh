#!/bin/bash
# br_qy.hip under max-memory-clause (the new default build): blind-rotate parity tests, then more
# machine-scheduler variants of it (build_variants/qx_*) against the in-tree library at B = 32768.
set -o pipefail
OUT=gpurun_out/${1:-r4p}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_pbs_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
bash tools/gpu_sched_ab.sh ${1:-r4p}/sab 2
