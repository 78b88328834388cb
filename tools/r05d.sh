set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_distributed.py -x -v -k "external_event or graph or data_parallel" --timeout 200 --timeout-method thread > gpurun_out/r05d_tests.log 2>&1 || { tail -40 gpurun_out/r05d_tests.log; exit 1; }
tail -12 gpurun_out/r05d_tests.log
REPS=3 bash tools/ab_env.sh NMGP_CHOL_LDS_KB 0 160
