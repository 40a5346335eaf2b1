#!/bin/bash
# Same-box A/B of the product build against variants (build_variants/NAME) on both blind-rotate
# kernels: latency kernel at B = 1 and 256, throughput kernel at B = 32768, classic and multi-bit
# (FHE_PROBE_MB=1).  usage: tools/ab_round.sh OUTFILE VARIANT...   (output under gpurun_out/)
set -o pipefail
OUT=$1; shift
for mb in 0 1; do
  for B in 1 256 32768; do
    R=5; [ $B = 32768 ] && R=3
    for v in fhe-sign_amd "$@"; do
      P=$v; [ $v != fhe-sign_amd ] && P=build_variants/$v
      FHE_PROBE_MB=$mb timeout -k 10 150 python3 tools/variant_probe.py $P $B $R >> $OUT 2>&1 || exit 2
    done
  done
done
