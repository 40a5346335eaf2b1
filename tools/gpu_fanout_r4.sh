#!/bin/bash
# config-5 fan-out projection (emulated ranks, per-rank replay; tools/fanout_projection.py) on the final tree
set -o pipefail
OUT=gpurun_out/${1:-fanout}
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/fanout_projection.py 1 2 4 8 > $OUT/fanout_projection.txt 2>&1 || { tail -20 $OUT/fanout_projection.txt; exit 1; }
cat $OUT/fanout_projection.txt
