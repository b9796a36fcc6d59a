# round 3: wide bf16 inference forward (variants/wide.so) against the 8-wave form, then fp32 200k (part)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
timeout -k 10 200 python3 tools/mlp_bench.py --dtype bf16 --M 786432 --reps 5 --rounds 4 --libs variants/base.so,variants/wide.so > gpurun_out/wide_mlp.json 2> gpurun_out/wide_mlp.log
r=$?; echo "mlp rc=$r"; cat gpurun_out/wide_mlp.json; if [ $r -ne 0 ]; then tail -5 gpurun_out/wide_mlp.log; exit $r; fi
for lib in base wide; do
  timeout -k 10 200 python3 tools/march_bench.py --dtype bf16 --lib variants/$lib.so --schedule 12x2_klow8_t0.9_g8 > gpurun_out/wide_march_$lib.json 2> gpurun_out/wide_march_$lib.log
  r=$?; echo "march $lib rc=$r"; cat gpurun_out/wide_march_$lib.json; if [ $r -ne 0 ]; then exit $r; fi
done
bash tools/gpu_psnr200k.sh fp32
