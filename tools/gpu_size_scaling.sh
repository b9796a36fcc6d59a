# Per-launch MLP kernel times at the coarse (262,144), fine (786,432) and merged (1,048,576) launch sizes of a step.
cd $GRAFT_REPO_ROOT
for dt in bf16 bf16x3f fp32; do for M in 262144 786432 1048576; do
  echo "$dt $M $(timeout -k 10 120 python3 tools/mlp_bench.py --libs nerf-replication_amd/nerf_amd/libnerf_amd.so --dtype $dt --M $M --rounds 3 2>/dev/null | tail -1)"
done; done
