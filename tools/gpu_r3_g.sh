# round 3: SIMD-partner stagger (finish delay of waves 4..7) variants, bf16 MLP kernels, interleaved
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for M in 786432; do
timeout -k 10 240 python3 tools/mlp_bench.py --dtype bf16 --M $M --reps 5 --rounds 4 --libs variants/base.so,nerf-replication_amd/nerf_amd/libnerf_amd.so,variants/fd7.so,variants/fd11.so > gpurun_out/stagger_$M.json 2> gpurun_out/stagger_$M.log
r=$?; echo "M=$M rc=$r"; cat gpurun_out/stagger_$M.json; if [ $r -ne 0 ]; then tail -5 gpurun_out/stagger_$M.log; exit $r; fi
done
