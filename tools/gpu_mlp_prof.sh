export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/mlp_bench.py > gpurun_out/mlpb.json 2>gpurun_out/mlpb.err && \
timeout -k 10 120 python tools/mlp_bench.py --M 262144 >> gpurun_out/mlpb.json 2>>gpurun_out/mlpb.err && \
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc1 -o p --output-format csv -- python3 tools/mlp_bench.py --reps 2 > gpurun_out/pmc1.log 2>&1
echo rc=$?
cat gpurun_out/mlpb.json
