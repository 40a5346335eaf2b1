#!/bin/bash
# PMC passes over one launch of the throughput kernel (pbs_probe at batch B), one counter group per
# rocprofv3 run (never combined with other trace domains).  usage: tools/pmc_passes.sh OUT B [mb]
# (mb: multi-bit keys).  Output under gpurun_out/OUT/<pass>/; summarise with tools/pmc_summary.py.
set -o pipefail
OUT=gpurun_out/${1:-pmc}; B=${2:-8192}
[ "$3" = "mb" ] && export FHE_PROBE_MB=1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="python3 tools/pbs_probe.py $B 1"
run() {  # name counters...
  local n=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$n -o run --output-format csv -- $P > $OUT/$n.log 2>&1
}
run fetch FETCH_SIZE || exit 1
run write WRITE_SIZE || exit 2
run l2 GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum || exit 3
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 4
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_VMEM_WR || exit 5
run ta TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum || exit 6
run ta2 TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum || exit 7
run tcp TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit 8
echo done
