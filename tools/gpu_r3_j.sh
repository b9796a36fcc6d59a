# round 3: the last part of the fp32 200k curve, then the N = 2 / 4 gloo rehearsal of the bench
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
bash tools/gpu_psnr200k.sh fp32 || exit $?
bash tools/gpu_r3_nrank.sh
