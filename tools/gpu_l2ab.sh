#!/bin/bash
# Same-box time + L2 A/B of throughput-kernel builds: the in-tree library (base) against every
# build_variants/qx_* (tools/build_variant.sh) at B = 32768, three interleaved rounds, then one
# FETCH_SIZE and one TCC hit/miss PMC pass per build (the key stream's L2 residency).
set -o pipefail
TAG=${1:-l2ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
bash tools/gpu_sched_ab.sh $TAG/sab 3 || exit 1
for V in base $(cd build_variants && ls -d qx_* 2>/dev/null); do
  for P in "FETCH_SIZE" "GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum"; do
    n=$(echo $P | cut -c1-5)
    timeout -k 10 180 rocprofv3 --pmc $P --kernel-trace -d $OUT/pmc_$V/$n -o run --output-format csv -- python3 tools/variant_probe.py build_variants/$V 32768 1 distinct > $OUT/pmc_$V.$n.log 2>&1 || exit 2
  done
done
echo l2ab-done
