#!/bin/bash
# SQ counters of the count kernel under DBSCAN_COUNT_ABLATE cases (timing/diagnostics only).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=gpurun_out/pmcab; rm -rf $OUT; mkdir -p $OUT
ARGS="--steps 2 --warmup 1 --no-cpu-baseline --no-profile"
G="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU"
G2="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT"
for a in ${CASES:-1 4}; do
  for g in 1 2; do
    [ $g = 1 ] && grp="$G" || grp="$G2"
    DBSCAN_COUNT_ABLATE=$a timeout -k 10 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/a$a/g$g -o run -- python3 bench.py $ARGS > $OUT/a$a.g$g.log 2>&1 || { echo "case $a failed"; tail -5 $OUT/a$a.g$g.log; exit 1; }
  done
  echo "ablate $a: $(python3 tools/pmc_agg.py $OUT/a$a | grep '^count_tile')"
done
