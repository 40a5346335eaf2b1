#!/bin/bash
# Round-5 check of the tree: smoke(), the -m gpu suite, the default bench line, then the bare
# `bench.py --gpus 2` rehearsal (self-launched ranks sharing the one GPU).  usage: tools/gpu_check_r5.sh TAG [skip_tests]
set -o pipefail
TAG=${1:-r5}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1 || { tail -20 $OUT/smoke.txt; exit 1; }
cat $OUT/smoke.txt
if [ -z "$2" ]; then
  timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 2; }
  tail -2 $OUT/gpu_tests.txt
fi
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms'],d.get('latency_level_ms'),{k:round(v['seconds'],4) for k,v in d['ops'].items()})"
timeout -k 10 900 python3 bench.py --gpus 2 --steps 3 --warmup 1 --no-multibit --no-cpu-baseline > $OUT/bench_gpus2.json 2> $OUT/bench_gpus2.err
echo "gpus2 rc=$?"
tail -5 $OUT/bench_gpus2.err
python3 -c "import json;d=json.load(open('$OUT/bench_gpus2.json'));print(d['n_gpus'],d['value'],d.get('fanout'))"
