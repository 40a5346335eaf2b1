#!/bin/bash
# Round-end check on the committed tree: smoke, the full GPU suite, then the default bench line.
set -o pipefail
OUT=gpurun_out/${1:-final}
mkdir -p $OUT
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 2; }
tail -2 $OUT/gpu_tests.txt
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms'],d.get('latency_level_ms'),{k:round(v['seconds'],4) for k,v in d['ops'].items()}, d['multibit']['value'], {k:round(v['seconds'],4) for k,v in d['multibit']['ops'].items()})"
