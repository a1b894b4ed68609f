#!/bin/bash
# Count-pass ablations (timing only; results are wrong by design):
#   DBSCAN_COUNT_ABLATE 0 full, 1 no neighbour counts, 2 no neighbour lists,
#   3 fused union without pair tests, 4 count alone (fused union off),
#   5 adjacent pair tests only, 6 no find-pruning of the distance-2 tests
set -o pipefail
mkdir -p gpurun_out
for a in ${CASES:-0 3 4 1}; do
  DBSCAN_COUNT_ABLATE=$a timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ca_$a.log 2>&1 || exit $?
  echo "ablate=$a $(python -c "import json; d=json.loads([l for l in open('gpurun_out/ca_$a.log') if l.startswith('{')][-1]); k=d['kernels_ms_per_step']; print(d['ms_per_step'], {n: k[n] for n in ('count', 'tile_union', 'quarter_init', 'edge_union') if n in k})")"
done
