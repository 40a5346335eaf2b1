#!/bin/bash
# A/B of build_variants/<NAME> against the in-tree library, interleaved runs of tools/variant_probe.py
# (B distinct encryptions).  usage: tools/gpu_variant_ab.sh TAG NAME [B] [rounds]
set -o pipefail
OUT=gpurun_out/${1:-vab}; NAME=$2; B=${3:-32768}; R=${4:-3}
mkdir -p $OUT
mkdir -p build_variants/base && rm -rf build_variants/base/fhe_sign build_variants/base/lib && cp -r fhe-sign_amd/fhe_sign fhe-sign_amd/lib build_variants/base/
for i in $(seq 1 $R); do
  for V in base $NAME; do
    timeout -k 10 180 python3 -u tools/variant_probe.py build_variants/$V $B 3 distinct >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 1; }
  done
done
cat $OUT/ab.txt
