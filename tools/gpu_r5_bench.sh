# Round-5 measurement call: the default bench line, its rocprof kernel stats, and the N=8 launcher
# rehearsal on the one-GPU box (gloo; bf16 so that 8 ranks' training stores fit one GPU's HBM).
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 900 python3 -u bench.py > gpurun_out/bench_r5.json 2> gpurun_out/bench_r5.err || { echo bench failed; tail -20 gpurun_out/bench_r5.err; exit 1; }
tail -c 600 gpurun_out/bench_r5.json
rm -rf gpurun_out/prof_r5
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r5 -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eager-baseline > gpurun_out/prof_r5.log 2>&1 || { echo prof failed; tail -20 gpurun_out/prof_r5.log; exit 1; }
find gpurun_out/prof_r5 -name "*stats*"
if [ "${1:-}" = "n8" ]; then
  NERF_BENCH_BACKEND=gloo timeout -k 10 900 python3 -u bench.py --gpus 8 --steps 3 --warmup 1 --no-second --dtype bf16 > gpurun_out/bench_n8_gloo.json 2> gpurun_out/bench_n8_gloo.err || { echo n8 failed; tail -30 gpurun_out/bench_n8_gloo.err; exit 1; }
  tail -c 400 gpurun_out/bench_n8_gloo.json
fi
