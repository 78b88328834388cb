#!/bin/bash
# MFMA-busy of the trailing-update SYRKs INSIDE factorizations, one PMC pass each:
#   stress: the M=4096 fp32 blocked potrf (gemm_big launches = its trailing SYRKs, k = 128)
#   ecog:   one ECoG-shaped training step (D=128, M=1024, 8385 batched factorizations; the recursive
#           chol_inv's Schur updates A22 -= L21 L21^T run as batched gemm_big SYRKs with k = 512, 256, 128)
# counters: SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE (own pass, no tracing domains)
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/syrkin
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/stress -o run -- python3 $R/tools/potrf_timeline.py > $OUT/stress.log 2>&1
timeout -s KILL 400 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $OUT/ecog -o run -- python3 $R/tools/ecog_bench.py train --steps 1 > $OUT/ecog.log 2>&1
cd $R
python3 tools/mfma_summary.py $(find $OUT/stress -name "*counter_collection.csv") $OUT/stress_mfma.json > /dev/null
python3 tools/mfma_summary.py $(find $OUT/ecog -name "*counter_collection.csv") $OUT/ecog_mfma.json > /dev/null
echo done
