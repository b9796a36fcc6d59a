# round 3: kernel trace of the default (one-pass, k_low growth) march
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/march_trace1
for dt in bf16 fp32; do
  timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/march_trace1/$dt -o m --output-format csv -- python3 tools/march_bench.py --dtype $dt --schedule 12x2_klow8_t0.9_g8 > gpurun_out/march_trace1_$dt.log 2>&1
  r=$?; echo "trace $dt rc=$r"; grep schedule gpurun_out/march_trace1_$dt.log; if [ $r -ne 0 ]; then exit $r; fi
done
