#!/bin/bash
# Register budget sweep of the tile/edge union kernels (DBSCAN_UNION_W: 6 default, 5, 7 waves/SIMD).
set -o pipefail
mkdir -p gpurun_out
for w in ${WS:-6 5 7}; do
  for d in "--noise 0.0" "--noise 0.2 --seed 2" "--points-per-gpu 20000000 --dense 8 --seed 3"; do
    DBSCAN_UNION_W=$w timeout -k 10 120 python bench.py --steps 10 --warmup 3 --no-cpu-baseline $d > gpurun_out/uw.log 2>&1 || exit $?
    echo "w=$w $d $(python -c "import json; d=json.loads([l for l in open('gpurun_out/uw.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print(d['ms_per_step'], k['tile_union'], k['edge_union'])")"
  done
done
