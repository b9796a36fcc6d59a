# Write-request shape of the bf16 training forward and dX stores: TCC_EA0_WRREQ (every
# write request to the fabric) against TCC_EA0_WRREQ_64B (the 64-byte ones); one pass, two TCC counters.
#   bash tools/gpu_pmc_writes.sh [DTYPE=bf16] [M=524288]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
DT=${1:-bf16}
M=${2:-524288}
O=gpurun_out/pmcw_$DT
rm -rf $O; mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum -d $O -o p --output-format csv -- \
  python3 tools/mlp_bench.py --dtype $DT --M $M --reps 2 > $O/run.log 2>&1
rc=$?
python3 tools/pmc_summary.py $O/p_counter_collection.csv > $O/summary.txt 2>&1
cat $O/summary.txt | head -40
exit $rc
