#!/bin/bash
# Count-kernel capacity x occupancy sweep (DBSCAN_COUNT_CAP: 0 = 1536 at 5 waves/SIMD, 1024 at 5,
# 2048 at 4); results identical, only the count time moves.
set -o pipefail
mkdir -p gpurun_out
for c in ${CAPS:-0 1024 2048}; do
  for d in "--noise 0.0" "--noise 0.2 --seed 2" "--points-per-gpu 20000000 --dense 8 --seed 3"; do
    DBSCAN_COUNT_CAP=$c timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $d > gpurun_out/cs.log 2>&1 || exit $?
    echo "cap=$c $d $(python -c "import json; d=json.loads([l for l in open('gpurun_out/cs.log') if l.startswith('{')][-1]); print(d['ms_per_step'], d['kernels_ms_per_step']['count'])")"
  done
done
