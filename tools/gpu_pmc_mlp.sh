# PMC passes over the MLP microbenchmark (each pass its own run): stalls, instruction mix, clock
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/pmcA -o p --output-format csv -- python3 tools/mlp_bench.py --reps 2 > gpurun_out/pmcA.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE GRBM_COUNT -d gpurun_out/pmcB -o p --output-format csv -- python3 tools/mlp_bench.py --reps 2 > gpurun_out/pmcB.log 2>&1 && \
timeout -s KILL 90 rocprofv3 --kernel-trace -d gpurun_out/pmcT -o p --output-format csv -- python3 tools/mlp_bench.py --reps 2 > gpurun_out/pmcT.log 2>&1
rc=$?
echo rc=$rc
exit $rc
