set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_engine.py tests/test_gpu_api.py tests/test_gpu_training_api.py tests/test_gpu_pair_shard.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eng_tests.log 2>&1
tail -2 gpurun_out/eng_tests.log
REPS=3 bash tools/ab_env.sh NMGP_SIDE3 0 1
