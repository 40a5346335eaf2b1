#!/bin/bash
# Interleaved same-box A/B of throughput-kernel variant builds (tools/build_variant.sh) against the product
# build: each run a fresh process (tools/qy2_probe.py).  usage: tools/kv_ab.sh ROUNDS KIND VARIANT...
set -u
R=$1; K=$2; shift 2
for r in $(seq 1 "$R"); do
  timeout -k 10 120 python -u tools/qy2_probe.py fhe-sign_amd "$K" 32768 3 || exit $?
  for v in "$@"; do timeout -k 10 120 python -u tools/qy2_probe.py "build_variants/$v" "$K" 32768 3 || exit $?; done
done
