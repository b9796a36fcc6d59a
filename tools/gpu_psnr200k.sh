# config 3 (200k steps x 4096 rays, PSNR every 10 epochs = 5000 steps) for one MLP dtype, continued
# across GPU calls: reads ckpt/psnr200k/<dtype>.pt if present, writes gpurun_out/psnr200k/
# usage: bash tools/gpu_psnr200k.sh <dtype> [check]
export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
DT=$1
mkdir -p gpurun_out/psnr200k
if [ "$2" = "check" ]; then  # resume exactness: 200 + 200 steps == 400 straight
  rm -rf /tmp/rs && mkdir -p /tmp/rs
  timeout -k 10 200 python3 -u tools/psnr_curve.py --dtypes $DT --steps 200 --every 100 --ckpt-out /tmp/rs/a > gpurun_out/psnr200k/check_a.log 2>&1 || exit 11
  timeout -k 10 200 python3 -u tools/psnr_curve.py --dtypes $DT --steps 400 --every 100 --ckpt-in /tmp/rs/a --ckpt-out /tmp/rs/b > gpurun_out/psnr200k/check_b.log 2>&1 || exit 12
  timeout -k 10 200 python3 -u tools/psnr_curve.py --dtypes $DT --steps 400 --every 100 --ckpt-out /tmp/rs/c > gpurun_out/psnr200k/check_c.log 2>&1 || exit 13
  python3 - <<'PY' > gpurun_out/psnr200k/check.json || exit 14
import json, torch
b = torch.load("/tmp/rs/b/DT.pt".replace("DT", __import__("os").environ.get("DT", "bf16")), weights_only=True)
c = torch.load("/tmp/rs/c/DT.pt".replace("DT", __import__("os").environ.get("DT", "bf16")), weights_only=True)
same_net = all(torch.equal(b["net"][k], c["net"][k]) for k in c["net"])
print(json.dumps({"resume_bit_exact_weights": same_net, "curve_b": b["curve"].tolist(), "curve_c": c["curve"].tolist()}))
PY
  cat gpurun_out/psnr200k/check.json
fi
CKIN=""
if [ -f ckpt/psnr200k/$DT.pt ]; then CKIN="--ckpt-in ckpt/psnr200k"; fi
timeout -k 10 1150 python3 -u tools/psnr_curve.py --dtypes $DT --steps 200000 --every 5000 $CKIN --ckpt-out gpurun_out/psnr200k --max-seconds ${PSNR_SECONDS:-960} > gpurun_out/psnr200k/run_$DT.log 2>&1
r=$?; tail -4 gpurun_out/psnr200k/run_$DT.log; exit $r
