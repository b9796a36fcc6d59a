export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
for l in variants/*.so; do timeout -k 10 120 python tools/grad_margin.py --lib $l >> gpurun_out/grad_margin.json 2>>gpurun_out/gm.err || exit $?; done
cat gpurun_out/grad_margin.json
