#!/bin/bash
# Same-box A/B of machine-scheduler builds (tools/build_variant.sh with EXTRA_FLAGS) against the
# in-tree library: throughput variants (qx_*) at B = 32768, latency variants (w_*) at B = 1 and 256.
# usage: tools/gpu_sched_ab.sh TAG ROUNDS
set -o pipefail
OUT=gpurun_out/${1:-sab}; R=${2:-2}
mkdir -p $OUT build_variants/base
rm -rf build_variants/base/fhe_sign build_variants/base/lib && cp -r fhe-sign_amd/fhe_sign fhe-sign_amd/lib build_variants/base/
run() { timeout -k 10 240 python3 -u tools/variant_probe.py build_variants/$1 $2 3 distinct >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }; }
for i in $(seq 1 $R); do
  for V in base $(cd build_variants && ls -d qx_* 2>/dev/null); do run $V 32768; done
  for B in 1 256; do
    for V in base $(cd build_variants && ls -d w_* 2>/dev/null); do run $V $B; done
  done
done
cat $OUT/ab.txt
