#!/bin/bash
# Round-end evidence in one GPU call: smoke, the default bench (config 2 with the CPU baseline and
# the end-to-end leg and the seam leg), the node path at N = 1 on config 3's per-GPU share, its
# one-rank RCCL rehearsal (--force-collectives), configs 3/4/5 per-GPU shares, config 5 itself
# through dbscan_train_node (phase trace), the node path's phase trace with RCCL forced, then
# tools/profile.sh (kernel trace + PMC passes).
# Each step under its own limit; the first failure ends the script.  NO_PROFILE=1: benches only;
# TAG names the profile summaries (gpurun_out/ev/profiles/<TAG>_*, copy them to profiles/).
set -o pipefail
mkdir -p gpurun_out/ev
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/ev/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ev/$name.log; exit $rc; }
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 400 python bench.py --steps 20 --warmup 5
run bench_node 300 python bench.py --node --config 3 --steps 10 --warmup 3
run bench_rccl 300 python bench.py --force-collectives --config 3 --steps 10 --warmup 3 --no-cpu-baseline
run bench_noise 300 python bench.py --config 3 --steps 10 --warmup 3 --no-cpu-baseline --no-seam
run bench_dense 300 python bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --no-seam
run bench_big 300 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 2 --no-seam
# config 5 itself (10^9 points) through the one-process whole-node entry, phase trace on stderr
DBSCAN_NODE_TRACE=1 run train_node_config5 400 python -u tools/train_node_probe.py 1e9 8
run node_phase_trace 300 python -u tools/node_phase_trace.py
grep -h '^{' gpurun_out/ev/bench_*.log | cut -c1-200
[ "${NO_PROFILE:-0}" = 1 ] && exit 0
# the raw traces exceed gpurun's 64 MiB return limit: summarize here, keep the summaries only
bash tools/profile.sh || exit 1
mkdir -p gpurun_out/ev/profiles
PROF_DEST=gpurun_out/ev/profiles python3 tools/pmc_summary.py gpurun_out/prof ${TAG:-round_ev} > gpurun_out/ev/pmc_summary.txt 2>&1 || exit 1
cp gpurun_out/prof/trace.log gpurun_out/ev/profile_trace.log
rm -rf gpurun_out/prof
# the default bench once more with this run's counters in place (profiles/pmc_traffic.json on the
# box is the snapshot's; the one just written is stamped with the running sources), so the
# committed default line carries roofline.traffic
cp gpurun_out/ev/profiles/pmc_traffic.json profiles/pmc_traffic.json || exit 1
run bench_default_traffic 400 python bench.py --steps 20 --warmup 5 --no-cpu-baseline
grep -h '"traffic"' gpurun_out/ev/bench_default_traffic.log | cut -c1-120 || true
