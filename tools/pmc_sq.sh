#!/bin/bash
# Diagnostic PMC passes (one counter group per pass) for the fit kernels on the bench workload.
#   bash tools/pmc_sq.sh            -> gpurun_out/pmcsq/p*/...; summarize with tools/pmc_agg.py
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcsq; rm -rf $OUT; mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-profile"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/p$i -o run -- python3 bench.py $ARGS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
  echo "pass $i ok"
done <<GROUPS
${PMC_GROUPS:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU
SQ_LEVEL_WAVES SQ_INST_LEVEL_VMEM SQ_INST_LEVEL_LDS SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_INSTS_SMEM
TCC_HIT_sum TCC_MISS_sum
TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr}
GROUPS
