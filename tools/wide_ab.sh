#!/bin/bash
# Same-box A/B of latency-kernel variants (built by tools/build_variant.sh ... br_wide) at the
# latency-level batches B = 1 and 256: the product build, then each variant, twice round.
# usage: tools/wide_ab.sh OUTFILE VARIANT...
set -o pipefail
OUT=$1; shift
for rep in 1 2; do
  for B in 1 256; do
    timeout -k 10 120 python3 tools/variant_probe.py fhe-sign_amd $B 5 >> $OUT 2>&1 || exit 2
    for v in "$@"; do
      timeout -k 10 120 python3 tools/variant_probe.py build_variants/$v $B 5 >> $OUT 2>&1 || exit 3
    done
  done
done
