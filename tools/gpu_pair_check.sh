set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_pair_shard.py tests/test_gpu_engine.py -x -v -s --timeout 200 --timeout-method thread > gpurun_out/pair_tests.log 2>&1
grep -E "PARITY|passed|failed" gpurun_out/pair_tests.log | tail -20
timeout -k 10 500 python -u tools/ecog_bench.py shard --world 8 --ranks 0,1,6,7 --steps 3 > gpurun_out/ecog_shard.log 2>&1
tail -5 gpurun_out/ecog_shard.log
