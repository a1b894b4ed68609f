set -o pipefail
mkdir -p gpurun_out/sab
for r in 1 2 3; do for v in head1 main; do
  lib=""; [ $v != main ] && lib=dbscan-on-spark_amd/lib_ab/$v/libdbscan_hip.so
  DBSCAN_LIB_PATH=$lib timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --e2e-steps 0 > gpurun_out/sab/$v.$r.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/sab/$v.$r.log; exit 1; }
  echo "$v $r done"
done; done
