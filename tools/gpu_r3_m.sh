# round 3: a second bf16 200k run from another seed (run-to-run PSNR spread of one precision)
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/psnr200k_s1
timeout -k 10 1150 python3 -u tools/psnr_curve.py --dtypes bf16 --steps 200000 --every 5000 --seed 1 --ckpt-out gpurun_out/psnr200k_s1 --max-seconds 1100 > gpurun_out/psnr200k_s1/run_bf16.log 2>&1
r=$?; tail -3 gpurun_out/psnr200k_s1/run_bf16.log; exit $r
