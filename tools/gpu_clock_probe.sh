#!/bin/bash
# Shader clock of the latency kernel at B = 1, 64, 256 (GRBM_GUI_ACTIVE summed over the 8 XCDs / kernel
# duration): is the B = 256 latency penalty the chip's clock under load?
set -o pipefail
OUT=gpurun_out/${1:-clock_r5}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for B in 1 64 256; do
  timeout -k 10 120 rocprofv3 --pmc GRBM_GUI_ACTIVE --kernel-trace -d $OUT/b$B -o run --output-format csv -- python3 tools/pbs_probe.py $B 3 > $OUT/b$B.log 2>&1 || exit 1
done
echo clock-done
