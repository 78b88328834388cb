set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_ecog.py tests/test_gpu_engine.py -x -q -k "big or ecog or rec or potrf or chol or hcp or pair" --timeout 300 --timeout-method thread > gpurun_out/r05ad_tests.log 2>&1 || { tail -30 gpurun_out/r05ad_tests.log; exit 1; }
tail -1 gpurun_out/r05ad_tests.log
timeout -k 10 200 ./tools/big8p_probe.x 512 1024 > gpurun_out/r05ad_big8p_probe.jsonl 2>&1 || { cat gpurun_out/r05ad_big8p_probe.jsonl; exit 1; }
cut -c1-160 gpurun_out/r05ad_big8p_probe.jsonl
timeout -k 10 240 python -u tools/big_probe.py > gpurun_out/r05ad_big_probe.jsonl 2>&1 || { tail -20 gpurun_out/r05ad_big_probe.jsonl; exit 1; }
grep variant gpurun_out/r05ad_big_probe.jsonl | cut -c1-110
bash tools/gpu_final_r05d.sh r05zg
