#!/bin/bash
# Same-box A/B of classic qy builds (tools/build_variant.sh) at mid level sizes, where a CU holds one or two
# workgroups, fresh process per run (tools/qy2_probe.py).  usage: tools/qy_mid_ab.sh VARIANT...
set -u
for r in 1 2; do
  for B in 300 384 512 768; do
    timeout -k 10 120 python -u tools/qy2_probe.py fhe-sign_amd 4 $B 3 || exit $?
    for v in "$@"; do timeout -k 10 120 python -u tools/qy2_probe.py "build_variants/$v" 4 $B 3 || exit $?; done
  done
done
