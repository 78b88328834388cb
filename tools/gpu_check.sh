#!/bin/bash
# One GPU-box pass: GPU parity tests, smoke, default bench line, then (optional) rocprof evidence.
# usage (from the repo root on the box): bash tools/gpu_check.sh [profile-prefix]
set -e
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1
tail -3 gpurun_out/gpu_tests.log
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke.log 2>&1
tail -1 gpurun_out/smoke.log
timeout -k 10 300 python -u bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
tail -1 gpurun_out/bench.json | cut -c1-600
if [ -n "$1" ]; then
  bash tools/profile_bench.sh "$1"
fi
