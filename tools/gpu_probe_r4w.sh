#!/bin/bash
# f64 / 32-bit issue probe (tools/fp64_issue_probe, built on the CPU side) and the latency-vs-throughput
# kernel sweep around the wide threshold (tools/lat_kinds.py) on the final qy build.
set -o pipefail
OUT=gpurun_out/${1:-r4w}
mkdir -p $OUT
timeout -k 10 120 ./tools/fp64_issue_probe > $OUT/issue_probe.txt 2>&1 || { tail -20 $OUT/issue_probe.txt; exit 1; }
cat $OUT/issue_probe.txt
timeout -k 10 300 python3 -u tools/lat_kinds.py --kinds wide,qy 3 128 256 320 384 512 640 768 > $OUT/lat_kinds.txt 2>&1 || { tail -20 $OUT/lat_kinds.txt; exit 2; }
cat $OUT/lat_kinds.txt
