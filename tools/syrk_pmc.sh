#!/bin/bash
# MFMA-busy evidence for the trailing-update SYRK (gemm_big_kernel) and the stress Cholesky:
#   pass 1: kernel trace + stats of tools/chol_stress.py (blocked potrf and chol+inv at M=4096)
#   pass 2: SQ_VALU_MFMA_BUSY_CYCLES + SQ_BUSY_CU_CYCLES + GRBM_GUI_ACTIVE over tools/syrk_probe.py (own pass)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/syrk
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 python3 $R/tools/syrk_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err
cat $OUT/probe.jsonl
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 $R/tools/chol_stress.py 4096 > $OUT/stress_trace.log 2>&1
grep "M=" $OUT/stress_trace.log
timeout -s KILL 120 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/pmc -o run -- python3 $R/tools/syrk_probe.py --reps 3 > $OUT/pmc.log 2>&1
python3 $R/tools/mfma_summary.py $OUT/pmc/run_counter_collection.csv $OUT/mfma_summary.json
echo done
