#!/bin/bash
# Round-3 pass I (fresh container): whole GPU suite incl. ECoG, default bench line, Cholesky A/B, rocprof evidence.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/r03i_suite.log 2>&1
rc=$?; tail -8 gpurun_out/r03i_suite.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r03i_bench.json 2> gpurun_out/r03i_bench.err
rc2=$?; tail -c 1500 gpurun_out/r03i_bench.json; [ $rc2 -ne 0 ] && { tail -20 gpurun_out/r03i_bench.err; exit $rc2; }
timeout -k 10 120 python -u tools/chol_ab.py 256:4:f64 256:1:f64 > gpurun_out/r03i_chol_ab.jsonl 2>&1 || exit $?
cat gpurun_out/r03i_chol_ab.jsonl
bash tools/profile_bench.sh r03i_pm25_bench > gpurun_out/r03i_prof.log 2>&1 || { tail -20 gpurun_out/r03i_prof.log; exit 5; }
ls gpurun_out
exit $rc
