# One parametrised GPU-box script (replaces the round-3 one-offs gpu_r3_[a-n].sh):
#   gpurun -- bash tools/gpu_run.sh STEP [STEP ...]
# Steps (each under its own time limit; the script stops at the first failure):
#   tests            the whole -m gpu suite
#   tests=EXPR       -m gpu tests selected by -k EXPR (+ for spaces)
#   file=PATH        -m gpu tests of one file
#   smoke            __graft_entry__.smoke()
#   bench            the default bench line (python bench.py)
#   benchq           a short bench (10 steps, no CPU / eager baselines)
#   nrank=N          bench.py --gpus N on this one GPU (gloo rehearsal of the launcher path)
#   rccl1            the RCCL (nccl backend) collective path at world size 1
#   prof             rocprofv3 --kernel-trace --stats of a short bench -> gpurun_out/prof/
#   pmc=DTYPE        PMC passes (traffic + stall counters) of the MLP kernels -> gpurun_out/pmc_DTYPE/
#   mlp=ARGS         tools/mlp_bench.py ARGS (comma-free; use + for spaces)
#   march=DTYPE      tools/march_bench.py --dtype DTYPE
#   ab=DTYPE         tools/step_ab.py --dtype DTYPE (whole-step A/B of the backward scheduling knobs)
#   abp=DTYPE        tools/step_ab.py --dtype DTYPE --configs one,noplan (the pack plan gather vs the direct repack)
#   abe=DTYPE        tools/step_ab.py --dtype DTYPE --configs one,events (cost of the per-kernel timing events)
#   abu=DTYPE        tools/step_ab.py --dtype DTYPE --configs one,unfused (the round-4 fused launches split again)
#   traffic=DTYPE    PMC FETCH_SIZE / WRITE_SIZE passes of a short bench -> gpurun_out/traffic_DTYPE.json
# Logs go to gpurun_out/<step>.log.
export TMPDIR=/tmp
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
PYT="python -u -m pytest -m gpu -v -s --timeout 300 --timeout-method thread"
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "[gpu_run] $name: $*"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local r=$?
  tail -4 "gpurun_out/$name.log"
  echo "[gpu_run] $name rc=$r"
  if [ $r -ne 0 ]; then
    grep -E "FAILED|Error" "gpurun_out/$name.log" | head -20
    exit $r
  fi
}
nm=0
for step in "$@"; do
  case "$step" in
    tests) run tests 1000 $PYT --maxfail=10 tests ;;
    tests=*) nm=$((nm + 1)); k=${step#tests=}; run "tests_k$nm" 900 $PYT --maxfail=10 tests -k "${k//+/ }" ;;
    file=*) f=${step#file=}; run "file_$(basename $f .py)" 900 $PYT --maxfail=10 "$f" ;;
    smoke) run smoke 180 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench) run bench 600 python3 -u bench.py ;;
    benchq) run benchq 400 python3 -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eager-baseline ;;
    nrank=*) n=${step#nrank=}; NERF_BENCH_BACKEND=gloo run "nrank$n" 700 python3 -u bench.py --gpus "$n" --steps 3 --warmup 1 ;;
    rccl1) run rccl1 200 python3 -u tools/rccl_probe.py ;;
    prof) rm -rf gpurun_out/prof
          run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- \
            python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-eager-baseline ;;
    pmc=*) run "pmc_${step#pmc=}" 900 bash tools/gpu_pmc_mlp.sh "${step#pmc=}" ;;
    traffic=*) dt=${step#traffic=}; rm -rf gpurun_out/tr_$dt
          B="python3 bench.py --dtype $dt --no-second --no-render --no-cpu-baseline --no-eager-baseline --steps 3 --warmup 1 --detail-steps 2"
          run "trF_$dt" 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/tr_$dt/F -o p --output-format csv -- $B
          run "trW_$dt" 300 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/tr_$dt/W -o p --output-format csv -- $B
          python3 tools/pmc_traffic.py gpurun_out/tr_$dt/F/p_counter_collection.csv gpurun_out/tr_$dt/W/p_counter_collection.csv $dt > gpurun_out/traffic_$dt.json || exit 1 ;;
    mlp=*) args=${step#mlp=}; nm=$((nm + 1)); run "mlp$nm" 600 python3 tools/mlp_bench.py ${args//+/ } ;;
    abe=*) run "abe_${step#abe=}" 600 python3 -u tools/step_ab.py --dtype "${step#abe=}" --configs one,events --rounds 7 ;;
    abu=*) run "abu_${step#abu=}" 600 python3 -u tools/step_ab.py --dtype "${step#abu=}" --configs one,unfused --rounds 7 ;;
    ab=*) run "ab_${step#ab=}" 600 python3 -u tools/step_ab.py --dtype "${step#ab=}" ;;
    abp=*) run "abp_${step#abp=}" 600 python3 -u tools/step_ab.py --dtype "${step#abp=}" --configs one,noplan --rounds 7 ;;
    march=*) run "march_${step#march=}" 400 python3 tools/march_bench.py --dtype "${step#march=}" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
