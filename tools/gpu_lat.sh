#!/bin/bash
# Latency-level kernels on the GPU: the blind-rotate parity tests (every kernel kind bit-identical),
# the latency sweep by kernel (tools/lat_kinds.py), the qyl variant builds (build_variants/qyl_*, made
# on the CPU side with tools/build_variant.sh: each without one of its three tunings) and a same-box
# qx/qy throughput A/B.  usage: tools/gpu_lat.sh TAG
set -o pipefail
OUT=gpurun_out/${1:-lat}
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest tests/test_pbs_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
timeout -k 10 300 python3 -u tools/lat_kinds.py 5 1 64 256 512 > $OUT/lat_kinds.txt 2>&1 || { tail -20 $OUT/lat_kinds.txt; exit 2; }
cat $OUT/lat_kinds.txt
for V in $(cd build_variants 2>/dev/null && ls -d qyl_* 2>/dev/null); do
  timeout -k 10 200 python3 -u tools/lat_kinds.py --pkg build_variants/$V --kinds qyl 5 1 256 >> $OUT/lat_variants.txt 2>&1 || { tail -20 $OUT/lat_variants.txt; exit 3; }
done
[ -f $OUT/lat_variants.txt ] && cat $OUT/lat_variants.txt
timeout -k 10 300 python3 -u tools/br_ab.py 32768 4 4 3 > $OUT/br_ab.txt 2>&1 || { tail -20 $OUT/br_ab.txt; exit 4; }
cat $OUT/br_ab.txt
