#!/bin/bash
# full -m gpu suite, the default bench line, then the config-5 fan-out projection (emulated ranks)
set -o pipefail
OUT=gpurun_out/${1:-r4f}
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 1; }
tail -2 $OUT/gpu_tests.txt
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['roofline']['frac'],{k:round(v['seconds'],4) for k,v in d['ops'].items()})"
timeout -k 10 600 python3 -u tools/fanout_projection.py 1 2 4 8 > $OUT/fanout_projection.txt 2>&1 || { tail -20 $OUT/fanout_projection.txt; exit 3; }
cat $OUT/fanout_projection.txt
