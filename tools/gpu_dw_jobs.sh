# per-job fp32 dW timing with the diagnostic build (variants/dwdiag.so, -DNERF_DW_DIAG=1)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
: > gpurun_out/dw_jobs.json
for dt in ${DW_DTYPES:-fp32}; do
for j in all 0 1 2 3 4 5 6 7 8 9; do
  if [ $j = all ]; then unset NERF_DW_ONLY_JOB; else export NERF_DW_ONLY_JOB=$j; fi
  echo "{\"job\": \"$j\", \"dtype\": \"$dt\", \"r\": $(timeout -k 10 120 python tools/mlp_bench.py --dtype $dt --libs variants/dwdiag.so --M 524288 --reps 5 --rounds 3 2>>gpurun_out/dw_jobs.err)}" >> gpurun_out/dw_jobs.json || exit 1
done
done
cat gpurun_out/dw_jobs.json
