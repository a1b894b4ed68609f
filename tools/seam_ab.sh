#!/bin/bash
# A/B of the seam leg (bench.py's per-call and per-partition timings) over library variants:
#   VARIANTS="base main" ROUNDS=3 bash tools/seam_ab.sh      (main: the in-tree library;
#   others: dbscan-on-spark_amd/lib_ab/<name>/libdbscan_hip.so from tools/build_ab.sh)
set -o pipefail
mkdir -p gpurun_out/sab
for r in $(seq 1 ${ROUNDS:-2}); do for v in ${VARIANTS:-main}; do
  lib=""; [ $v != main ] && lib=dbscan-on-spark_amd/lib_ab/$v/libdbscan_hip.so
  DBSCAN_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 > gpurun_out/sab/$v.$r.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/sab/$v.$r.log; exit 1; }
  python3 - "$v" gpurun_out/sab/$v.$r.log <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[2]) if l.startswith("{")][-1])
s = d["seam"]
pc = " ".join(f"{k}:{v['host_us']}/{v['device_us']}" for k, v in s["per_call"].items())
t = s["train"]
print(f"{sys.argv[1]:8s} {pc} pp1 {t['per_partition_calls']['us_per_partition']} "
      f"pp4 {t['per_partition_calls_4_threads']['us_per_partition']}")
PY
done; done
