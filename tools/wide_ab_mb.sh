#!/bin/bash
set -o pipefail
OUT=$1; shift
export FHE_PROBE_MB=1
for rep in 1 2; do
  for B in 1 256; do
    timeout -k 10 120 python3 tools/variant_probe.py fhe-sign_amd $B 5 >> $OUT 2>&1 || exit 2
    for v in "$@"; do
      timeout -k 10 120 python3 tools/variant_probe.py build_variants/$v $B 5 >> $OUT 2>&1 || exit 3
    done
  done
done
