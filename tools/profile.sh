#!/bin/bash
# rocprofv3 evidence for the bench workload (bench.py defaults unless BENCH_ARGS is set):
#   1 kernel trace + stats;  2 FETCH_SIZE;  3 WRITE_SIZE (they cannot share a pass on gfx950);
#   4-6 SQ counter groups (8 SQ counters per pass at most: MI355X_MICROARCH.md §PMC slots).
# Each pass is its own bench run under its own time limit; the first failure ends the script.
#   bash tools/profile.sh && python tools/pmc_summary.py gpurun_out/prof rNN
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
OUT=${PROF_OUT:-gpurun_out/prof}
rm -rf $OUT; mkdir -p $OUT
ARGS="${BENCH_ARGS:---steps 5 --warmup 2} --no-cpu-baseline --e2e-steps 0 --no-seam"
python3 -c "import bench; print(bench.src_stamp())" > $OUT/src_sha || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1 || { echo "trace failed"; tail -20 $OUT/trace.log; exit 1; }
echo "trace ok"
i=0
while read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $grp --output-format csv -d $OUT/pmc$i -o run -- python3 bench.py $ARGS --no-profile > $OUT/pmc$i.log 2>&1 || { echo "pmc pass $i ($grp) failed"; tail -5 $OUT/pmc$i.log; exit 1; }
  echo "pmc pass $i ok"
done <<GROUPS
FETCH_SIZE
WRITE_SIZE
SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU
SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32
SQ_INSTS_LDS SQ_INSTS_VALU_INT32 SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS
GROUPS
