#!/bin/bash
# Same-box A/B of blind-rotate builds (tools/build_variant.sh, EXTRA_FLAGS = scheduler strategies):
# default quad and pair kernels against the variants named on the command line (pair variants: p_*).
set -o pipefail
for rep in 1 2; do
  timeout -k 10 120 python tools/variant_probe.py fhe-sign_amd 8192 4 >> gpurun_out/sched_ab.txt 2>&1 || exit 2
  FHE_BR_KERNEL=2 timeout -k 10 120 python tools/variant_probe.py fhe-sign_amd 8192 4 >> gpurun_out/sched_ab.txt 2>&1 || exit 3
  for v in "$@"; do
    case $v in p_*) export FHE_BR_KERNEL=2;; *) unset FHE_BR_KERNEL;; esac
    timeout -k 10 120 python tools/variant_probe.py build_variants/$v 8192 4 >> gpurun_out/sched_ab.txt 2>&1 || exit 4
  done
  unset FHE_BR_KERNEL
done
