set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -v -k "pair_streaming" --timeout 200 --timeout-method thread > gpurun_out/r05e_tests.log 2>&1 || { tail -60 gpurun_out/r05e_tests.log; exit 1; }
tail -10 gpurun_out/r05e_tests.log
