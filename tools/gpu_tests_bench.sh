#!/bin/bash
# The GPU tests named on the command line, then the default bench line (the round's check after a radix
# change).  usage: tools/gpu_tests_bench.sh TAG tests/test_a.py [tests/test_b.py ...]
set -o pipefail
OUT=gpurun_out/${1:?tag}
shift
mkdir -p $OUT
timeout -k 10 600 python3 -u -m pytest "$@" -x -v --timeout 300 --timeout-method thread > $OUT/tests.txt 2>&1 || { tail -40 $OUT/tests.txt; exit 2; }
tail -3 $OUT/tests.txt
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms'],d.get('latency_level_ms'),{k:round(v['seconds'],4) for k,v in d['ops'].items()}, d['multibit']['value'], {k:round(v['seconds'],4) for k,v in d['multibit']['ops'].items()})"
