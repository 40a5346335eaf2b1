#!/bin/bash
# Same-box A/B at the bench batch (32768): default quad vs the pair kernel (default build and the
# variants named on the command line, built by tools/build_variant.sh).
set -o pipefail
for rep in 1 2; do
  timeout -k 10 150 python tools/variant_probe.py fhe-sign_amd 32768 3 >> gpurun_out/batch_ab.txt 2>&1 || exit 2
  for v in "$@"; do
    FHE_BR_KERNEL=2 timeout -k 10 150 python tools/variant_probe.py build_variants/$v 32768 3 >> gpurun_out/batch_ab.txt 2>&1 || exit 3
  done
done
