#!/bin/bash
# qy default: stagger variants A/B (build_variants/qy_stag*, tools/build_variant.sh) against the
# in-tree library at B = 32768, then the full -m gpu suite and the default bench line.
set -o pipefail
OUT=gpurun_out/${1:-r4m}
mkdir -p $OUT build_variants/base
rm -rf build_variants/base/fhe_sign build_variants/base/lib && cp -r fhe-sign_amd/fhe_sign fhe-sign_amd/lib build_variants/base/
for i in 1 2; do
  for V in base $(cd build_variants && ls -d qy_* 2>/dev/null); do
    timeout -k 10 240 python3 -u tools/variant_probe.py build_variants/$V 32768 3 distinct >> $OUT/stagger_ab.txt 2>&1 || { tail -20 $OUT/stagger_ab.txt; exit 1; }
  done
done
cat $OUT/stagger_ab.txt
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $OUT/gpu_tests.txt 2>&1 || { tail -30 $OUT/gpu_tests.txt; exit 2; }
tail -2 $OUT/gpu_tests.txt
timeout -k 10 600 python3 bench.py > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 3; }
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['roofline']['frac'],d.get('latency_level_ms'),{k:round(v['seconds'],4) for k,v in d['ops'].items()})"
