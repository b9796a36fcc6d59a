# rocprof kernel stats of the grid march (bf16, trained fixture net) for the current build
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/march_prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/march_prof -o m --output-format csv -- python3 tools/march_bench.py --dtype bf16 > gpurun_out/march_prof.log 2>&1 || exit 1
grep -h "march\|fwd_kernel" gpurun_out/march_prof/*kernel_stats.csv | cut -d, -f1-5
