# round 3: finish-delay sweep (fp32 and bf16 MLP kernels, interleaved builds, outputs compared)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for dt in fp32 bf16; do
  timeout -k 10 300 python3 tools/mlp_bench.py --dtype $dt --M 524288 --reps 3 --rounds 4 --libs variants/base.so,variants/fd1.so,variants/fd2.so,variants/fd5.so > gpurun_out/fd_$dt.json 2> gpurun_out/fd_$dt.log
  r=$?; echo "$dt rc=$r"; cat gpurun_out/fd_$dt.json; if [ $r -ne 0 ]; then tail -5 gpurun_out/fd_$dt.log; exit $r; fi
done
