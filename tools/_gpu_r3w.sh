set -o pipefail
mkdir -p gpurun_out/w/profiles
PROF_OUT=gpurun_out/prof5 BENCH_ARGS="--config 5 --steps 2 --warmup 1" bash tools/profile.sh || exit 1
PROF_DEST=gpurun_out/w/profiles python3 tools/pmc_summary.py gpurun_out/prof5 round3_m_config5 --no-json > gpurun_out/w/sum_c5.txt 2>&1 || exit 1
cp gpurun_out/prof5/trace.log gpurun_out/w/trace_c5.log; rm -rf gpurun_out/prof5
