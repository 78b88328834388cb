#!/bin/bash
# Round-3 pass Y: evidence for the shipped code -- whole GPU suite, default bench line, rocprofv3 kernel
# trace + FETCH/WRITE passes (profile_bench.sh), MFMA-busy pass (pm25_pmc.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/r03y_suite.log 2>&1
rc=$?; tail -4 gpurun_out/r03y_suite.log
[ $rc -gt 1 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r03y_bench.json 2> gpurun_out/r03y_bench.err
rc2=$?; [ $rc2 -ne 0 ] && { tail -20 gpurun_out/r03y_bench.err; exit $rc2; }
python -c "
import json;d=json.loads(open('gpurun_out/r03y_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['cholesky'], d['hcp_train']['it_per_s'], d['ecog_train']['s_per_step'], d['api_path']['device_with_predict_Y'], d['cholesky_stress']['potrf_ms'])"
bash tools/profile_bench.sh r03y_pm25_bench > gpurun_out/r03y_prof.log 2>&1 || { tail -20 gpurun_out/r03y_prof.log; exit 5; }
bash tools/pm25_pmc.sh > gpurun_out/r03y_pmc.log 2>&1 || { tail -20 gpurun_out/r03y_pmc.log; exit 6; }
python tools/step_timeline.py $(find gpurun_out/prof/trace -name "*kernel_trace.csv") > gpurun_out/r03y_step_timeline.txt 2>&1
head -3 gpurun_out/r03y_step_timeline.txt
exit $rc
