#!/bin/bash
# r5: default bench line on the compat carry-count chain + the config-5 fan-out projection
set -o pipefail
OUT=gpurun_out/${1:-r5d}
mkdir -p $OUT
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms'],d.get('latency_level_ms'),{k:round(v['seconds'],4) for k,v in d['ops'].items()}, d['multibit']['value'], {k:round(v['seconds'],4) for k,v in d['multibit']['ops'].items()})"
timeout -k 10 900 python3 -u tools/fanout_projection.py 1 2 4 8 > $OUT/fanout_projection.txt 2>&1 || { tail -20 $OUT/fanout_projection.txt; exit 1; }
tail -30 $OUT/fanout_projection.txt
