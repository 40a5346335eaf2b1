#!/bin/bash
# Same-box A/B of machine-scheduler builds (tools/build_variant.sh with EXTRA_FLAGS) against the
# in-tree library: throughput variants (qx_*) at B = 32768, latency variants (w_*) at B = 1 and 256,
# multi-bit throughput variants (mb_*, br_quad.hip) at B = 32768 on multi-bit keys.
# usage: tools/gpu_sched_ab.sh TAG ROUNDS
set -o pipefail
OUT=gpurun_out/${1:-sab}; R=${2:-2}
mkdir -p $OUT build_variants/base
rm -rf build_variants/base/fhe_sign build_variants/base/lib && cp -r fhe-sign_amd/fhe_sign fhe-sign_amd/lib build_variants/base/
run() { timeout -k 10 240 python3 -u tools/variant_probe.py build_variants/$1 $2 3 distinct >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }; }
runmb() { FHE_PROBE_MB=1 timeout -k 10 240 python3 -u tools/variant_probe.py build_variants/$1 $2 3 distinct >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }; }
for i in $(seq 1 $R); do
  for V in base $(cd build_variants && ls -d qx_* 2>/dev/null); do run $V 32768; done
  if ls -d build_variants/w_* > /dev/null 2>&1; then
    for B in 1 256; do
      for V in base $(cd build_variants && ls -d w_* 2>/dev/null); do run $V $B; done
    done
    if [ -n "${SAB_MB_LAT:-}" ]; then  # the multi-bit latency kernel too
      for B in 1 256; do
        for V in base $(cd build_variants && ls -d w_* 2>/dev/null); do runmb $V $B; done
      done
    fi
  fi
  if ls -d build_variants/mb_* > /dev/null 2>&1; then
    for V in base $(cd build_variants && ls -d mb_* 2>/dev/null); do runmb $V 32768; done
  fi
done
cat $OUT/ab.txt
