#!/bin/bash
# One parameterised GPU-box runner (replaces the per-pass tools/gpu_r03*.sh scripts of round 3).
# usage (from the repo root, on the GPU box):  bash tools/gpu_run.sh <tag> <step> [<step> ...]
# steps:
#   suite      the whole -m gpu suite                      -> gpurun_out/<tag>_suite.log
#   bench      default bench.py line                       -> gpurun_out/<tag>_bench.json
#   prof       rocprofv3 kernel trace + FETCH/WRITE passes -> gpurun_out/<tag>_pm25_bench_*  (tools/profile_bench.sh)
#   pmc        MFMA-busy pass of the PM2.5 step            -> gpurun_out/pm25pmc/            (tools/pm25_pmc.sh)
#   timeline   step timeline from the prof kernel trace    -> gpurun_out/<tag>_step_timeline.txt
#   stress     stress potrf kernel trace + MFMA pass       -> gpurun_out/stress/             (tools/stress_trace.sh)
#   train      HCP / ECoG training kernel breakdowns      -> gpurun_out/<tag>_{hcp,ecog}_train_kernels.json
#   potrf      stress potrf tests, timing, trace, MFMA    -> gpurun_out/<tag>_stress_*     (tools/stress_potrf.sh)
#   n2         bench.py's N = 2 path rehearsed with two gloo ranks sharing cuda:0
#   n4         the same with four gloo ranks
# Every GPU step runs under its own timeout and the script stops at the first failing step.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
TAG=$1; shift
run() {  # run <name> <cmd...>: the caller's `|| { ...; exit 1; }` stops the script on failure
  local name=$1; shift
  echo "== $name: $*" >&2
  "$@"
  local rc=$?
  [ $rc -ne 0 ] && echo "== $name failed rc=$rc" >&2
  return $rc
}
for step in "$@"; do
  case $step in
    suite)
      run suite timeout -k 10 900 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread \
        > gpurun_out/${TAG}_suite.log 2>&1 || { tail -30 gpurun_out/${TAG}_suite.log; exit 1; }
      tail -3 gpurun_out/${TAG}_suite.log ;;
    bench)
      run bench timeout -k 10 500 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
        || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
      tail -1 gpurun_out/${TAG}_bench.json | cut -c1-600 ;;
    prof)
      run prof bash tools/profile_bench.sh ${TAG}_pm25_bench > gpurun_out/${TAG}_prof.log 2>&1 \
        || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; } ;;
    pmc)
      run pmc bash tools/pm25_pmc.sh > gpurun_out/${TAG}_pmc.log 2>&1 || { tail -20 gpurun_out/${TAG}_pmc.log; exit 1; } ;;
    timeline)
      python tools/step_timeline.py $(find gpurun_out/prof/trace -name "*kernel_trace.csv") > gpurun_out/${TAG}_step_timeline.txt 2>&1
      head -3 gpurun_out/${TAG}_step_timeline.txt ;;
    stress)
      run stress bash tools/stress_trace.sh > gpurun_out/${TAG}_stress.log 2>&1 || { tail -20 gpurun_out/${TAG}_stress.log; exit 1; } ;;
    potrf)
      run potrf bash tools/stress_potrf.sh $TAG > gpurun_out/${TAG}_potrf.log 2>&1 || { tail -30 gpurun_out/${TAG}_potrf.log; exit 1; }
      tail -25 gpurun_out/${TAG}_potrf.log ;;
    train)
      run train bash tools/train_trace.sh $TAG > gpurun_out/${TAG}_train.log 2>&1 || { tail -20 gpurun_out/${TAG}_train.log; exit 1; }
      tail -28 gpurun_out/${TAG}_train.log ;;
    quick)
      # the round's new GPU tests first (a fault here stops the script before the long steps)
      run quick timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -q -x --timeout 200 \
        --timeout-method thread -k "${QUICK_K:-potrf}" > gpurun_out/${TAG}_quick.log 2>&1 \
        || { tail -30 gpurun_out/${TAG}_quick.log; exit 1; }
      tail -3 gpurun_out/${TAG}_quick.log ;;
    n2|n4)
      n=${step#n}
      # never the measured configuration: gloo ranks sharing one GPU, shapes small enough for n ranks per card
      run $step env NMGP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 20 --warmup 5 \
        --no-breakdown --pair-D 32 --elbo-D 32 > gpurun_out/${TAG}_bench_n${n}_rehearsal.json \
        2> gpurun_out/${TAG}_bench_n${n}_rehearsal.err || { tail -20 gpurun_out/${TAG}_bench_n${n}_rehearsal.err; exit 1; }
      tail -1 gpurun_out/${TAG}_bench_n${n}_rehearsal.json | cut -c1-600 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps done"
