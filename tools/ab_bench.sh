#!/bin/bash
# A/B the library variants built by tools/build_ab.sh on one GPU box, interleaved ROUNDS times:
#   VARIANTS="base new" ROUNDS=3 BENCH_ARGS="..." bash tools/ab_bench.sh
# "main" is the in-tree library.  Prints ms_per_step and the top kernels of every run (KERNELS="a b":
# those kernels instead).
set -o pipefail
mkdir -p gpurun_out/ab
ARGS="${BENCH_ARGS:---steps 20 --warmup 5} --no-cpu-baseline --e2e-steps 0"
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $VARIANTS; do
    lib=""
    [ "$v" != main ] && lib="dbscan-on-spark_amd/lib_ab/$v/libdbscan_hip.so"
    DBSCAN_LIB_PATH=$lib timeout -k 10 200 python bench.py $ARGS > gpurun_out/ab/$v.$r.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/ab/$v.$r.log; exit 1; }
    python3 - "$v" "gpurun_out/ab/$v.$r.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
k = d["kernels_ms_per_step"]
import os
want = os.environ.get("KERNELS", "").split()
top = ", ".join(f"{a}={b:.3f}" for a, b in (list(k.items())[:8] if not want else
                                           [(w, k.get(w, float("nan"))) for w in want]))
cnt = "+".join(f"{k.get(a, 0):.3f}" for a in ("count32", "count_wave", "count_tiny", "count_tiny16", "big_count"))
print(f"{sys.argv[1]:10s} {d['ms_per_step']:.4f} ms  k={d['config']['clusters']}  count {cnt}  {top}")
PY
  done
done
