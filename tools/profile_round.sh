#!/bin/bash
# Profiling session (run on the GPU box via gpurun).  Kernel trace + stats of the exact bench
# command whose roofline line is reported, a trace of the ops legs, then separate PMC passes
# (never combined with other trace domains) over one launch of the throughput kernel (B=8192) and
# one of the latency kernel (B=256).  Output under gpurun_out/$1; summarise with
# tools/pmc_summary.py gpurun_out/$1.
set -o pipefail
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ops > $OUT/bench_under_trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_ops -o run --output-format csv -- python3 tools/ops_timing.py > $OUT/ops_under_trace.log 2>&1 || exit 2
for B in 8192 256; do
  P="python3 tools/pbs_probe.py $B 1"
  timeout -k 10 200 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch_$B -o run --output-format csv -- $P > $OUT/pmc_fetch_$B.log 2>&1 || exit 3
  timeout -k 10 200 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write_$B -o run --output-format csv -- $P > $OUT/pmc_write_$B.log 2>&1 || exit 4
  timeout -k 10 200 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --kernel-trace -d $OUT/pmc_sq1_$B -o run --output-format csv -- $P > $OUT/pmc_sq1_$B.log 2>&1 || exit 5
  timeout -k 10 200 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR --kernel-trace -d $OUT/pmc_sq2_$B -o run --output-format csv -- $P > $OUT/pmc_sq2_$B.log 2>&1 || exit 6
  timeout -k 10 200 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum --kernel-trace -d $OUT/pmc_l2_$B -o run --output-format csv -- $P > $OUT/pmc_l2_$B.log 2>&1 || exit 7
done
find $OUT -name "*.csv" | head -80
