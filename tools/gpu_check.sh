#!/bin/bash
# GPU check of the current tree (run via gpurun): the -m gpu suite (optionally a subset), then the
# default bench line.  usage: tools/gpu_check.sh TAG [pytest selection...]
set -o pipefail
TAG=${1:-chk}; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
SEL=${@:-tests}
timeout -k 10 900 python3 -u -m pytest $SEL -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 1; }
tail -3 $OUT/gpu_tests.txt
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 2; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['roofline']['frac'],{k:round(v['seconds'],4) for k,v in d['ops'].items()})"
