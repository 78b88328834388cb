#!/bin/bash
# Round evidence pass on the GPU box (one call): default bench line, PM2.5 rocprofv3 kernel trace + FETCH /
# WRITE passes (tools/profile_bench.sh), MFMA-busy pass (tools/pm25_pmc.sh), PM2.5 step timeline
# (tools/timeline.sh), stress potrf timeline and its MFMA-busy pass.  Every GPU step has its own time limit
# and the chain stops at the first failure.  usage: bash tools/gpu_evidence.sh <prefix e.g. r02d>
set -e
P=${1:?prefix}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/ev
timeout -k 10 300 python -u bench.py > gpurun_out/ev/bench.json 2> gpurun_out/ev/bench.err
bash tools/profile_bench.sh ${P}_pm25_bench
bash tools/pm25_pmc.sh
cp gpurun_out/pm25pmc/pm25_mfma.json gpurun_out/ev/${P}_pm25_mfma.json
bash tools/timeline.sh $P
cp gpurun_out/tl_$P/timeline.txt gpurun_out/ev/${P}_pm25_step_timeline.txt
OUT=$R/gpurun_out/ev/stress
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/trace -o run -- python3 $R/tools/potrf_timeline.py 4096 > $OUT/trace.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- python3 $R/tools/potrf_timeline.py 4096 > $OUT/pmc.log 2>&1
cd $R
python3 tools/potrf_timeline.py --show $(find $OUT/trace -name "*kernel_trace.csv") > gpurun_out/ev/${P}_stress_potrf_timeline.txt
python3 tools/mfma_summary.py $(find $OUT/pmc -name "*counter_collection.csv") gpurun_out/ev/${P}_stress_potrf_mfma_util.json > /dev/null
echo evidence done
