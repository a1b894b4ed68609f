#!/bin/bash
# Round-end evidence in one GPU call: smoke, the default bench (config 2 with the CPU baseline and
# the end-to-end leg), the node path at N = 1 on config 3's per-GPU share, configs 4 and 5
# per-GPU shares, then tools/profile.sh (kernel trace + PMC passes).
# Each step under its own limit; the first failure ends the script.
set -o pipefail
mkdir -p gpurun_out/ev
run() {  # name, limit, command...
  local name=$1 lim=$2; shift 2
  timeout -k 10 $lim "$@" > gpurun_out/ev/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; [ $rc -eq 0 ] || { tail -5 gpurun_out/ev/$name.log; exit $rc; }
}
run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
run bench_default 400 python bench.py --steps 20 --warmup 5
run bench_node 300 python bench.py --node --steps 10 --warmup 3 --points-per-gpu 12500000 --noise 0.2 --seed 2
run bench_noise 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --points-per-gpu 12500000 --noise 0.2 --seed 2
run bench_dense 300 python bench.py --steps 5 --warmup 2 --no-cpu-baseline --points-per-gpu 50000000 --dense 8 --seed 3
run bench_big 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --e2e-steps 2 --points-per-gpu 125000000 --noise 0.2 --seed 4
grep -h '^{' gpurun_out/ev/bench_*.log | cut -c1-200
bash tools/profile.sh
