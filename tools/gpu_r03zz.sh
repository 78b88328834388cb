#!/bin/bash
# Round-3 pass ZZ (final): evidence for the shipped code -- whole GPU suite, default bench line, rocprofv3 kernel
# trace + FETCH/WRITE passes (profile_bench.sh), MFMA-busy pass (pm25_pmc.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -q -rf --timeout 400 --timeout-method thread > gpurun_out/r03zz_suite.log 2>&1
rc=$?; tail -4 gpurun_out/r03zz_suite.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py > gpurun_out/r03zz_bench.json 2> gpurun_out/r03zz_bench.err
rc2=$?; [ $rc2 -ne 0 ] && { tail -20 gpurun_out/r03zz_bench.err; exit $rc2; }
python -c "
import json;d=json.loads(open('gpurun_out/r03zz_bench.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['cholesky'], d['hcp_train']['it_per_s'], d['ecog_train']['s_per_step'], d['api_path']['device_with_predict_Y'], d['cholesky_stress']['potrf_ms'])"
bash tools/profile_bench.sh r03zz_pm25_bench > gpurun_out/r03zz_prof.log 2>&1 || { tail -20 gpurun_out/r03zz_prof.log; exit 5; }
bash tools/pm25_pmc.sh > gpurun_out/r03zz_pmc.log 2>&1 || { tail -20 gpurun_out/r03zz_pmc.log; exit 6; }
python tools/step_timeline.py $(find gpurun_out/prof/trace -name "*kernel_trace.csv") > gpurun_out/r03zz_step_timeline.txt 2>&1
head -3 gpurun_out/r03zz_step_timeline.txt
# bench.py's N = 2 path rehearsed with gloo ranks sharing cuda:0 (DP step with the all-reduce, KL-sharded ELBO
# and pair-sharded legs at D = 32 so that two ranks fit one GPU); never the measured configuration
NMGP_DIST_BACKEND=gloo timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 20 --warmup 5 --no-breakdown --pair-D 32 --elbo-D 32 > gpurun_out/r03zz_bench_n2_rehearsal.json 2> gpurun_out/r03zz_bench_n2_rehearsal.err
rc3=$?; tail -1 gpurun_out/r03zz_bench_n2_rehearsal.json | cut -c1-800; [ $rc3 -ne 0 ] && tail -20 gpurun_out/r03zz_bench_n2_rehearsal.err
exit $rc
