#!/bin/bash
# Round-5 final evidence, part B: rocprofv3 passes of the final code (PM2.5 kernel trace + FETCH / WRITE, PM2.5
# MFMA-busy, in-factorization SYRK MFMA-busy (stress + ECoG), stress HBM traffic, HCP / ECoG kernel breakdowns),
# copied into profiles/ (the bench line promotes only profiles whose code_hash matches), then the default bench line.
set -e
TAG=${1:-r05z}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
bash tools/profile_bench.sh ${TAG}_pm25_bench
bash tools/pm25_pmc.sh
python3 tools/mfma_summary.py $(find gpurun_out/pm25pmc/mfma -name "*counter_collection.csv") gpurun_out/${TAG}_pm25_mfma.json --by-grid > /dev/null
bash tools/syrk_inside_pmc.sh
python3 tools/mfma_summary.py $(find gpurun_out/syrkin/stress -name "*counter_collection.csv") gpurun_out/${TAG}_stress_potrf_mfma_util.json --by-grid > /dev/null
python3 tools/mfma_summary.py $(find gpurun_out/syrkin/ecog -name "*counter_collection.csv") gpurun_out/${TAG}_ecog_step_mfma_util.json --by-grid > /dev/null
bash tools/stress_hbm.sh $TAG
bash tools/train_trace.sh $TAG
bash tools/train_pmc.sh $TAG
cp gpurun_out/${TAG}_hcp_train_traffic.json gpurun_out/${TAG}_ecog_train_traffic.json profiles/
cp gpurun_out/${TAG}_pm25_bench_summary.json gpurun_out/${TAG}_pm25_bench_kernel_stats.csv gpurun_out/${TAG}_pm25_mfma.json \
   gpurun_out/${TAG}_stress_potrf_mfma_util.json gpurun_out/${TAG}_ecog_step_mfma_util.json gpurun_out/${TAG}_stress_potrf_hbm.json \
   gpurun_out/${TAG}_hcp_train_kernels.json gpurun_out/${TAG}_ecog_train_kernels.json profiles/
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
tail -1 gpurun_out/${TAG}_bench.json | cut -c1-300
