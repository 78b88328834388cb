#!/bin/bash
# MFMA-busy of every kernel of the PM2.5 bench step (gemm_kernel<double> and
# chol_inv2_kernel), one PMC pass (no tracing domains), summarised per (kernel, grid) by
# tools/mfma_summary.py --by-grid.  Under counter collection the dispatches are serialised, so
# avg_us is the kernel alone, not its time inside the overlapped graph.
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pm25pmc
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
ARGS="--steps 10 --warmup 2 --no-breakdown --no-cpu-baseline --no-stress --no-elbo --no-api --no-hcp --no-ecog --no-kron"
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/mfma -o run -- python3 $R/bench.py $ARGS > $OUT/mfma.log 2>&1
cd $R
python3 tools/mfma_summary.py $(find $OUT/mfma -name "*counter_collection.csv") $OUT/pm25_mfma.json --by-grid > $OUT/pm25_mfma.txt
echo done
