#!/bin/bash
# PMC passes (issue, address unit, L1) over one kernel variant built by tools/build_variant.sh,
# one counter group per rocprofv3 run.  usage: tools/pmc_variant.sh OUT build_variants/NAME B [mb]
set -o pipefail
OUT=gpurun_out/$1; PKG=$2; B=${3:-8192}
[ "$4" = "mb" ] && export FHE_PROBE_MB=1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
P="python3 tools/variant_probe.py $PKG $B 1"
run() {  # name counters...
  local n=$1; shift
  timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace -d $OUT/$n -o run --output-format csv -- $P > $OUT/$n.log 2>&1
}
run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM || exit 2
run ta2 TA_TA_BUSY_sum TA_BUFFER_WAVEFRONTS_sum || exit 3
run tcp TCP_PENDING_STALL_CYCLES_sum TCP_READ_TAGCONFLICT_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum || exit 4
echo done
