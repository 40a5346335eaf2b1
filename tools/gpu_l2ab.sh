#!/bin/bash
# Same-box time + L2 A/B of qy builds: build_variants/qx_a (max-memory-clause only), qx_b (+ key
# slices at the top of the step), base = in-tree (+ untwist loads after the second barrier, post-RA
# scheduler off); then one FETCH_SIZE and one TCC hit/miss pass per build at B = 32768; plus the
# latency kernel's key-prefetch variant (build_variants/w_kpre) at B = 1 and 256.
set -o pipefail
TAG=${1:-l2ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
bash tools/gpu_sched_ab.sh $TAG/sab 3 || exit 1
for V in base qx_a qx_b; do
  for P in "FETCH_SIZE" "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
    n=$(echo $P | cut -c1-5)
    timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace -d $OUT/pmc_$V/$n -o run --output-format csv -- python3 tools/variant_probe.py build_variants/$V 32768 1 distinct > $OUT/pmc_$V.$n.log 2>&1 || exit 2
  done
done
echo l2ab-done
