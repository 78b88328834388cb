#!/bin/bash
# Round-3 pass S: PARITY lines of the engine / ECoG / HCP tests (printed with -s) for DESIGN's table.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_ecog.py -q -s --timeout 400 --timeout-method thread > gpurun_out/r03s_parity.log 2>&1
rc=$?; grep -E "PARITY|passed|failed" gpurun_out/r03s_parity.log | cut -c1-400
exit $rc
