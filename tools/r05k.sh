set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -q -k "potrf" --timeout 200 --timeout-method thread > gpurun_out/r05k_tests.log 2>&1 || { tail -40 gpurun_out/r05k_tests.log; exit 1; }
tail -2 gpurun_out/r05k_tests.log
timeout -k 10 120 python tools/potrf_ab.py 4096 2048 > gpurun_out/r05k_potrf_ab.json 2> gpurun_out/r05k_potrf_ab.err || { tail -20 gpurun_out/r05k_potrf_ab.err; exit 1; }
cat gpurun_out/r05k_potrf_ab.json
