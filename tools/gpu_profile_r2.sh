# rocprofv3 evidence for bench.py (round 2): kernel trace + stats of the full bench (fp32
# headline + bf16x3 and bf16 lines), then FETCH_SIZE and WRITE_SIZE passes per dtype (each its own run),
# then the LDS / MFMA counters of the MLP kernels (fp32), then smoke.
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/prof_r2
rm -rf $OUT && mkdir -p $OUT
run() { echo "[$(date +%T)] $*" >> $OUT/progress.log; }
run trace
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o bench --output-format csv -- python3 bench.py --no-cpu-baseline --no-eager-baseline > $OUT/bench_under_rocprof.log 2>$OUT/bench_under_rocprof.err || exit 1
for dt in fp32 bf16x3 bf16; do
  run fetch $dt
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch_$dt -o fetch --output-format csv -- python3 bench.py --dtype $dt --no-second --steps 2 --warmup 1 --detail-steps 1 --no-cpu-baseline --no-eager-baseline --no-render > $OUT/fetch_$dt.log 2>&1 || exit 2
  run write $dt
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d $OUT/write_$dt -o write --output-format csv -- python3 bench.py --dtype $dt --no-second --steps 2 --warmup 1 --detail-steps 1 --no-cpu-baseline --no-eager-baseline --no-render > $OUT/write_$dt.log 2>&1 || exit 3
done
run pmc lds
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $OUT/pmc_lds -o p --output-format csv -- python3 tools/mlp_bench.py --dtype fp32 --M 524288 --reps 2 > $OUT/pmc_lds.log 2>&1 || exit 4
run pmc stall
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU -d $OUT/pmc_stall -o p --output-format csv -- python3 tools/mlp_bench.py --dtype fp32 --M 524288 --reps 2 > $OUT/pmc_stall.log 2>&1 || exit 5
run smoke
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 6
run done
