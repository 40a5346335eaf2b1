#!/bin/bash
# r5: full GPU suite + smoke, then the rocprof kernel trace / PMC passes of tools/profile_round.sh
set -o pipefail
TAG=${1:-r5e}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 2; }
tail -2 $OUT/gpu_tests.txt
bash tools/profile_round.sh $TAG/prof
