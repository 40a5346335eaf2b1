#!/bin/bash
# multi-bit blind rotation on br_qy.hip (FHE_MB_QY=1): bit-identity test, then a same-box A/B against
# br_quad.hip at B = 32768 on multi-bit keys, three interleaved rounds; PMC L2 check of both.
set -o pipefail
OUT=gpurun_out/${1:-mbqy}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 python3 -u -m pytest tests/test_pbs_gpu.py -m gpu -k "multibit_qy" -x -v --timeout 250 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -30 $OUT/tests.txt; exit 1; }
tail -2 $OUT/tests.txt
for i in 1 2 3; do
  FHE_PROBE_MB=1 timeout -k 10 240 python3 -u tools/variant_probe.py fhe-sign_amd 32768 3 distinct >> $OUT/ab.txt 2>&1 || { tail -20 $OUT/ab.txt; exit 2; }
  FHE_PROBE_MB=1 FHE_MB_QY=1 timeout -k 10 240 python3 -u tools/variant_probe.py fhe-sign_amd 32768 3 distinct 2>&1 | sed 's/^fhe-sign_amd/qy_mb/' >> $OUT/ab.txt || { tail -20 $OUT/ab.txt; exit 3; }
done
cat $OUT/ab.txt
