#!/bin/bash
# Same-box A/B of kernel variants built by tools/build_variant.sh (round-3 scheduler, phase-E, barrier
# and layout experiments; results in profiles/r3/*_ab_*.txt): the first variant's bit-exactness
# (tests/test_pbs_gpu.py against its library), then variant_probe timings of the product and every
# variant, twice, at the given batches.
# usage (GPU box): tools/sched_ab.sh OUTFILE "B1 B2 ..." VARIANT...   (FHE_PROBE_MB=1 for multi-bit keys)
set -o pipefail
O=$1; BS=$2; shift 2
FHE_ROCM_LIB=$PWD/build_variants/$1/lib/libfhe_rocm.so timeout -k 10 300 python -u -m pytest tests/test_pbs_gpu.py -x -q --timeout 120 --timeout-method thread >> $O 2>&1 || exit 3
for r in 1 2; do
  for B in $BS; do
    R=5; [ $B -ge 8192 ] && R=3
    for v in fhe-sign_amd "$@"; do
      P=$v; [ $v != fhe-sign_amd ] && P=build_variants/$v
      timeout -k 10 150 python3 tools/variant_probe.py $P $B $R >> $O 2>&1 || exit 2
    done
  done
done
