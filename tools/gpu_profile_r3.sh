# rocprofv3 evidence for bench.py (round 3): the default bench line, kernel trace + stats of the
# full bench, FETCH_SIZE and WRITE_SIZE passes per dtype (each its own run), MFMA/stall counters
# of the bf16 inference forward (the march's MLP).  Progress in gpurun_out/prof_r3/progress.log.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof_r3
rm -rf $OUT && mkdir -p $OUT
run() { echo "[$(date +%T)] $*" >> $OUT/progress.log; }
run bench
timeout -k 10 500 python3 -u bench.py > $OUT/bench_line.json 2> $OUT/bench_line.err || exit 1
run trace
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --no-cpu-baseline --no-eager-baseline > $OUT/bench_under_rocprof.json 2>$OUT/bench_under_rocprof.err || exit 2
for dt in fp32 bf16x3 bf16; do
  run fetch $dt
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$dt -o fetch --output-format csv -- python3 bench.py --dtype $dt --no-second --steps 2 --warmup 1 --detail-steps 1 --no-cpu-baseline --no-eager-baseline --no-render > $OUT/fetch_$dt.log 2>&1 || exit 3
  run write $dt
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$dt -o write --output-format csv -- python3 bench.py --dtype $dt --no-second --steps 2 --warmup 1 --detail-steps 1 --no-cpu-baseline --no-eager-baseline --no-render > $OUT/write_$dt.log 2>&1 || exit 4
done
run pmc stall bf16
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/pmc_stall_bf16 -o p --output-format csv -- python3 tools/mlp_bench.py --dtype bf16 --M 786432 --reps 2 > $OUT/pmc_stall_bf16.log 2>&1 || exit 5
run pmc clock bf16
timeout -s KILL 90 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_VALU_MFMA_COEXEC_CYCLES -d $OUT/pmc_clock_bf16 -o p --output-format csv -- python3 tools/mlp_bench.py --dtype bf16 --M 786432 --reps 2 > $OUT/pmc_clock_bf16.log 2>&1 || exit 6
run done
