#!/bin/bash
# Counter passes over one tune.py run (one variant, one element), for
# kernel diagnosis: issue/stall mix (SQ) and L2 / fabric requests (TCC).
# Each counter set is its own rocprofv3 --pmc pass (no tracing domains).
# Usage (GPU box): tools/pmc_kernel.sh <out> <workload> <element> [variant] [sets, e.g. 1,2]
set -euo pipefail
OUT=$1; WL=$2; EL=$3; VAR=${4:-base}; SETS=${5:-1,2,3,4}
export TMPDIR=/tmp TUNE_ELEMENT=$EL
mkdir -p "$OUT"
CMD="python3 tools/tune.py --workload $WL --variants $VAR --rounds 1 --launches 2"
SET1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU"
SET2="SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_SMEM"
SET3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"
SET4="TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE"
for i in ${SETS//,/ }; do
  eval "set=\$SET$i"
  timeout -s KILL 300 rocprofv3 --pmc $set --output-format csv -d "$OUT/p$i" -o run -- $CMD > "$OUT/p$i.log" 2>&1
done
python3 tools/pmc_table.py "$OUT" "$OUT/summary.json" > "$OUT/summary.txt"
