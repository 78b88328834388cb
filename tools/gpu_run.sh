#!/bin/bash
# The one parameterised GPU-box runner (round 6: replaces the per-round tools/r05*.sh and gpu_final_*.sh recipes).
# usage (from the repo root, on the GPU box):  bash tools/gpu_run.sh <tag> <step> [<step> ...]
# steps:
#   quick      tests/test_gpu_primitives.py -k "$QUICK_K" (the round's new kernels first)
#   suite      the whole -m gpu suite                          -> gpurun_out/<tag>_suite.log
#   smoke      __graft_entry__.smoke()                          -> gpurun_out/<tag>_smoke.log
#   bench      default bench.py line                           -> gpurun_out/<tag>_bench.json
#   prof       rocprofv3 kernel trace + FETCH/WRITE passes of the PM2.5 bench -> gpurun_out/<tag>_pm25_bench_*
#   pmc        MFMA-busy pass of the PM2.5 step                -> gpurun_out/<tag>_pm25_mfma.json
#   timeline   PM2.5 step timeline (kernel trace of a graphed run) -> gpurun_out/<tag>_pm25_step_timeline.txt
#   potrf      stress potrf tests, timing, trace, MFMA pass    -> gpurun_out/<tag>_stress_potrf_*
#   syrkin     MFMA-busy of the SYRKs inside the stress and ECoG factorizations -> gpurun_out/<tag>_{stress_potrf,ecog_step}_mfma_util.json
#   hbm        stress factorization FETCH / WRITE passes       -> gpurun_out/<tag>_stress_potrf_hbm.json
#   train      HCP / ECoG training kernel breakdowns           -> gpurun_out/<tag>_{hcp,ecog}_train_kernels.json
#   trainpmc   HCP / ECoG FETCH / WRITE and MFMA-busy passes   -> gpurun_out/<tag>_{hcp,ecog}_train_traffic.json
#   publish    copy the tag's summaries into profiles/ (the bench line promotes only code_hash-matched profiles)
#   n2 | n4    bench.py's N > 1 path rehearsed with gloo ranks sharing cuda:0 (never the measured configuration)
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
PM25_ARGS="--no-cpu-baseline --no-stress --no-elbo --no-api --no-hcp --no-ecog --no-kron"
for step in "$@"; do
  case $step in
    quick)
      run quick timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -q -x --timeout 200 \
        --timeout-method thread -k "${QUICK_K:-potrf}" > gpurun_out/${TAG}_quick.log 2>&1 \
        || { tail -30 gpurun_out/${TAG}_quick.log; exit 1; }
      tail -3 gpurun_out/${TAG}_quick.log ;;
    suite)
      run suite timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread \
        > gpurun_out/${TAG}_suite.log 2>&1 || { tail -30 gpurun_out/${TAG}_suite.log; exit 1; }
      tail -3 gpurun_out/${TAG}_suite.log ;;
    smoke)
      run smoke timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 \
        || { tail -20 gpurun_out/${TAG}_smoke.log; exit 1; }
      tail -2 gpurun_out/${TAG}_smoke.log ;;
    bench)
      run bench timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err \
        || { tail -20 gpurun_out/${TAG}_bench.err; exit 1; }
      tail -1 gpurun_out/${TAG}_bench.json | cut -c1-600 ;;
    prof)
      run prof bash tools/profile_bench.sh ${TAG}_pm25_bench > gpurun_out/${TAG}_prof.log 2>&1 \
        || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; } ;;
    pmc)
      OUT=$R/gpurun_out/pm25pmc_$TAG; mkdir -p $OUT
      (cd /tmp && export TMPDIR=/tmp && run pmc timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES \
        SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/mfma -o run -- python3 $R/bench.py --steps 10 \
        --warmup 2 --no-breakdown $PM25_ARGS > $OUT/mfma.log 2>&1) || { tail -20 $OUT/mfma.log; exit 1; }
      python3 tools/mfma_summary.py $(find $OUT/mfma -name "*counter_collection.csv") gpurun_out/${TAG}_pm25_mfma.json \
        --by-grid > /dev/null ;;
    timeline)
      OUT=$R/gpurun_out/tl_$TAG; mkdir -p $OUT
      (cd /tmp && export TMPDIR=/tmp && run timeline timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv \
        -d $OUT -o run -- python3 $R/bench.py --steps 20 --warmup 5 --no-breakdown $PM25_ARGS > $OUT/b.json \
        2> $OUT/err.log) || { tail -20 $OUT/err.log; exit 1; }
      python3 tools/step_timeline.py $(find $OUT -name "*kernel_trace.csv" | head -1) 1 \
        > gpurun_out/${TAG}_pm25_step_timeline.txt
      head -1 gpurun_out/${TAG}_pm25_step_timeline.txt ;;
    potrf)
      run potrf bash tools/stress_potrf.sh $TAG > gpurun_out/${TAG}_potrf.log 2>&1 || { tail -30 gpurun_out/${TAG}_potrf.log; exit 1; }
      tail -25 gpurun_out/${TAG}_potrf.log ;;
    syrkin)
      run syrkin bash tools/syrk_inside_pmc.sh > gpurun_out/${TAG}_syrkin.log 2>&1 || { tail -20 gpurun_out/${TAG}_syrkin.log; exit 1; }
      python3 tools/mfma_summary.py $(find gpurun_out/syrkin/stress -name "*counter_collection.csv") \
        gpurun_out/${TAG}_stress_potrf_mfma_util.json --by-grid > /dev/null
      python3 tools/mfma_summary.py $(find gpurun_out/syrkin/ecog -name "*counter_collection.csv") \
        gpurun_out/${TAG}_ecog_step_mfma_util.json --by-grid > /dev/null ;;
    hbm)
      run hbm bash tools/stress_hbm.sh $TAG > gpurun_out/${TAG}_hbm.log 2>&1 || { tail -20 gpurun_out/${TAG}_hbm.log; exit 1; } ;;
    train)
      run train bash tools/train_trace.sh $TAG > gpurun_out/${TAG}_train.log 2>&1 || { tail -20 gpurun_out/${TAG}_train.log; exit 1; }
      tail -4 gpurun_out/${TAG}_train.log ;;
    trainpmc)
      run trainpmc bash tools/train_pmc.sh $TAG > gpurun_out/${TAG}_trainpmc.log 2>&1 \
        || { tail -20 gpurun_out/${TAG}_trainpmc.log; exit 1; } ;;
    publish)
      for f in pm25_bench_summary.json pm25_bench_kernel_stats.csv pm25_mfma.json pm25_step_timeline.txt \
               stress_potrf_mfma_util.json ecog_step_mfma_util.json stress_potrf_hbm.json stress_potrf_timeline.txt \
               hcp_train_kernels.json ecog_train_kernels.json hcp_train_traffic.json ecog_train_traffic.json \
               suite.log smoke.log; do
        [ -f gpurun_out/${TAG}_$f ] && cp gpurun_out/${TAG}_$f profiles/
      done
      [ -f gpurun_out/${TAG}_bench.json ] && tail -1 gpurun_out/${TAG}_bench.json > profiles/${TAG}_pm25_bench_default.json
      ls profiles | grep "^${TAG}_" ;;
    n2|n4)
      n=${step#n}
      run $step env NMGP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 \
        --nproc-per-node $n --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 20 --warmup 5 \
        --no-breakdown --pair-D 32 --elbo-D 32 ${DP_MODE:+--dp-allreduce $DP_MODE} \
        > gpurun_out/${TAG}_bench_n${n}_rehearsal.json 2> gpurun_out/${TAG}_bench_n${n}_rehearsal.err \
        || { tail -20 gpurun_out/${TAG}_bench_n${n}_rehearsal.err; exit 1; }
      tail -1 gpurun_out/${TAG}_bench_n${n}_rehearsal.json | cut -c1-600 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "== all steps done"
