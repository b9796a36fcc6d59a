# PMC passes over the MLP microbenchmark, each pass its own run (rocprofv3 does not split
# counters over passes): A stalls / MFMA busy, B LDS / instruction mix / clock (GRBM), F HBM
# reads, W HBM writes.   bash tools/gpu_pmc_mlp.sh [DTYPE=bf16] [M=786432]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
DT=${1:-bf16}
M=${2:-786432}
LIB=${3:-}   # (an alternative build: tools/mlp_bench.py --lib)
O=gpurun_out/pmc_$DT${LIB:+_$(basename $LIB .so)}
rm -rf $O; mkdir -p $O
B="python3 tools/mlp_bench.py --dtype $DT --M $M --reps 2 ${LIB:+--lib $LIB}"
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU -d $O/A -o p --output-format csv -- $B > $O/A.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT -d $O/B -o p --output-format csv -- $B > $O/B.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d $O/F -o p --output-format csv -- $B > $O/F.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d $O/W -o p --output-format csv -- $B > $O/W.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/T -o p --output-format csv -- $B > $O/T.log 2>&1
rc=$?
echo rc=$rc
find $O -name "*.csv" | head -20
exit $rc
