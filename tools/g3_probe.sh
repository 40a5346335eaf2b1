#!/bin/bash
# Grouping-3 cost estimate: the multi-bit kernels with a grouping-3 step's shape
# (n/3 steps, 7 key patterns per step; timing only, wrong numbers) against the grouping-2 product
# kernels, same box: latency level (wide, B = 1 / 256) and throughput (quad, B = 32768).
# Variants: tools/build_variant.sh wide_g7 (-DWMB7, br_wide), quad_g7 (-DQMB7 -DQMB_D=1, br_quad),
# quad_g2d1 (-DQMB_D=1).  usage: tools/g3_probe.sh OUTFILE
set -o pipefail
OUT=$1
export FHE_PROBE_MB=1
for B in 1 256; do
  for v in fhe-sign_amd build_variants/wide_g7; do
    timeout -k 10 120 python3 tools/variant_probe.py $v $B 5 >> $OUT 2>&1 || exit 2
  done
done
for v in fhe-sign_amd build_variants/quad_g7 build_variants/quad_g2d1; do
  timeout -k 10 200 python3 tools/variant_probe.py $v 32768 3 >> $OUT 2>&1 || exit 3
done
