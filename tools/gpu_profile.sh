# rocprofv3 evidence for bench.py: kernel trace + stats, then FETCH_SIZE and WRITE_SIZE passes
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof
rm -rf $OUT && mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_under_rocprof.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o fetch --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render > $OUT/fetch.log 2>&1 && \
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o write --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-render > $OUT/write.log 2>&1
[ $? -eq 0 ] && timeout -k 10 300 python3 bench.py > $OUT/bench_plain.log 2>&1
rc=$?
echo rc=$rc
find $OUT -name "*.csv" | head -20
tail -1 $OUT/bench_under_rocprof.log
exit $rc
