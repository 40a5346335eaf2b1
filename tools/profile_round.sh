#!/bin/bash
# Profiling session (run on the GPU box via gpurun).  Kernel trace + stats of the exact bench
# command whose roofline lines are reported (classic headline and the multi-bit variant), a trace of
# the ops legs, then separate PMC passes (never combined with other trace domains) over one launch
# of the throughput kernel (B=32768, the bench batch) and one of the latency kernel (B=256), classic and multi-bit.
# Output under gpurun_out/$1; summarise with tools/pmc_summary.py gpurun_out/$1 profiles/rN/...json
set -o pipefail
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-ops > $OUT/bench_under_trace.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace_ops -o run --output-format csv -- python3 tools/ops_timing.py > $OUT/ops_under_trace.log 2>&1 || exit 2
for kind in cl mb; do
  if [ $kind = mb ]; then export FHE_PROBE_MB=1; else unset FHE_PROBE_MB; fi
  for B in 32768 256; do
    P="python3 tools/pbs_probe.py $B 1"
    D=$OUT/pmc_${kind}_$B
    run() { local n=$1; shift; timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace -d $D/$n -o run --output-format csv -- $P > $D.$n.log 2>&1; }
    mkdir -p $D
    run fetch FETCH_SIZE || exit 3
    run write WRITE_SIZE || exit 4
    run l2 GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum || exit 5
    run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 6
    run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR || exit 7
    run ta TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum || exit 8
    run tcp TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit 9
  done
done
echo profile-done
