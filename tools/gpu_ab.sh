#!/bin/bash
# quick same-box A/B of the classic throughput kernels (tools/br_ab.py), output under gpurun_out/TAG
set -o pipefail
OUT=gpurun_out/${1:-ab}
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/br_ab.py ${2:-32768} ${3:-4} > $OUT/br_ab.txt 2>&1; rc=$?
cat $OUT/br_ab.txt | tail -3
exit $rc
