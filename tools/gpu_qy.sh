#!/bin/bash
# br_qy.hip on the GPU: the throughput-kernel parity tests, a same-box qx/qy A/B at B = 32768, then the
# machine-scheduler / barrier-cost variants (tools/gpu_sched_ab.sh, one round).  usage: tools/gpu_qy.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-qy}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_pbs_gpu.py tests/test_kernel_resources.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
timeout -k 10 300 python3 -u tools/br_ab.py 32768 6 4 3 > $OUT/br_ab.txt 2>&1 || { tail -20 $OUT/br_ab.txt; exit 2; }
cat $OUT/br_ab.txt
tools/gpu_sched_ab.sh ${1:-qy}/sab 1
