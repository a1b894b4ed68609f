set -o pipefail
mkdir -p gpurun_out/n
S=gpurun_out/n/profiles
mkdir -p $S
bash tools/profile.sh || exit 1
PROF_DEST=$S python3 tools/pmc_summary.py gpurun_out/prof round3_k > gpurun_out/n/sum_c2.txt 2>&1 || exit 1
cp gpurun_out/prof/trace.log gpurun_out/n/trace_c2.log; rm -rf gpurun_out/prof
PROF_OUT=gpurun_out/prof5 BENCH_ARGS="--config 5 --steps 2 --warmup 1 --no-seam" bash tools/profile.sh || exit 1
PROF_DEST=$S python3 tools/pmc_summary.py gpurun_out/prof5 round3_k_config5 --no-json > gpurun_out/n/sum_c5.txt 2>&1 || exit 1
cp gpurun_out/prof5/trace.log gpurun_out/n/trace_c5.log; rm -rf gpurun_out/prof5
DBSCAN_NODE_TRACE=1 DBSCAN_TEST_FULL_SCALE=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k config5_full_size_vs_oracle -s -v --timeout 580 --timeout-method thread > gpurun_out/n/c5.log 2>&1
rc=$?; echo "c5 rc=$rc"; tail -5 gpurun_out/n/c5.log; exit $rc
