#!/bin/bash
# Stress configuration (BASELINE.json configs[4], one SPD M=4096 fp32 matrix) on the GPU box:
#   1. the blocked-potrf parity tests, 2. graph-replayed timing (tools/potrf_ab.py),
#   3. rocprofv3 kernel trace of one factorization -> per-launch timeline (tools/potrf_timeline.py --show),
#   4. one PMC pass (SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE, no tracing domains) ->
#      MFMA-busy per (kernel, grid) (tools/mfma_summary.py --by-grid).
# usage: bash tools/stress_potrf.sh <tag>     outputs gpurun_out/<tag>_stress_*
set -e
TAG=${1:-r04}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stress_$TAG
mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -q -k "potrf_blocked" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 120 python tools/potrf_ab.py 4096 2048 > $OUT/potrf_ab.json 2> $OUT/potrf_ab.err || { tail -20 $OUT/potrf_ab.err; exit 1; }
cat $OUT/potrf_ab.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/potrf_timeline.py > $OUT/trace.log 2>&1
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- python3 $R/tools/potrf_timeline.py > $OUT/pmc.log 2>&1
cd $R
python3 tools/potrf_timeline.py --show $(find $OUT/trace -name "*kernel_trace.csv") > gpurun_out/${TAG}_stress_potrf_timeline.txt
tail -1 gpurun_out/${TAG}_stress_potrf_timeline.txt
python3 tools/mfma_summary.py $(find $OUT/pmc -name "*counter_collection.csv") gpurun_out/${TAG}_stress_potrf_mfma_util.json --by-grid > gpurun_out/${TAG}_stress_potrf_mfma_util.txt
cat gpurun_out/${TAG}_stress_potrf_mfma_util.txt | head -40
