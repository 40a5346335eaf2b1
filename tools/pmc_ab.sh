#!/bin/bash
# PMC A/B of the classic throughput kernels (br_quad = 1, br_qx = 3) at batch B, one counter group per
# rocprofv3 run (never combined with other trace domains).  usage: tools/pmc_ab.sh OUT [B]
set -o pipefail
OUT=gpurun_out/${1:-pmcab}; B=${2:-32768}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for K in 1 3; do
  export FHE_PROBE_BR=$K
  P="python3 tools/pbs_probe.py $B 1"
  D=$OUT/k$K
  mkdir -p $D
  run() { local n=$1; shift; timeout -k 10 120 rocprofv3 --pmc "$@" --kernel-trace -d $D/$n -o run --output-format csv -- $P > $D.$n.log 2>&1; }
  run sq1 SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU || exit 1
  run sq2 SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_WR || exit 2
  run l2 GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum || exit 3
done
echo pmc-ab-done
