#!/bin/bash
# Same-box A/B of an issue-priority window in a throughput kernel variant (tools/build_variant.sh) against
# the product, at several level sizes, fresh process per run (tools/qy2_probe.py).
# usage: tools/qy_prio_ab.sh VARIANT KIND [mb]
set -u
V=$1; K=$2; MB=${3:-}
for r in 1 2 3; do
  for B in 512 1536 32768; do
    timeout -k 10 120 python -u tools/qy2_probe.py fhe-sign_amd "$K" $B 3 $MB || exit $?
    timeout -k 10 120 python -u tools/qy2_probe.py "build_variants/$V" "$K" $B 3 $MB || exit $?
  done
done
