#!/bin/bash
# HBM traffic of the stress factorization (configs[4]): FETCH_SIZE and WRITE_SIZE in two separate PMC passes of
# tools/potrf_timeline.py (no tracing domains), summarised by tools/stress_hbm.py -> gpurun_out/<tag>_stress_potrf_hbm.json
set -e
TAG=${1:-r05}
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/stresshbm_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 $R/tools/potrf_timeline.py > $OUT/fetch.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 $R/tools/potrf_timeline.py > $OUT/write.log 2>&1
cd $R
python3 tools/stress_hbm.py $(find $OUT/fetch -name "*counter_collection.csv") $(find $OUT/write -name "*counter_collection.csv") gpurun_out/${TAG}_stress_potrf_hbm.json
