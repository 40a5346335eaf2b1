#!/bin/bash
# Same-box A/B of throughput-kernel variants (built by tools/build_variant.sh ... br_qy) at the bench's
# batch (32768 distinct encryptions): the product build, then each variant, three times round.
# usage: tools/qy_ab.sh OUTFILE VARIANT...
set -o pipefail
OUT=$1; shift
for rep in 1 2 3; do
  timeout -k 10 180 python3 tools/variant_probe.py fhe-sign_amd 32768 3 distinct >> $OUT 2>&1 || exit 2
  for v in "$@"; do
    timeout -k 10 180 python3 tools/variant_probe.py build_variants/$v 32768 3 distinct >> $OUT 2>&1 || exit 3
  done
done
