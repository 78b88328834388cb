set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_ecog.py -x -q -k "big or ecog or rec" --timeout 300 --timeout-method thread > gpurun_out/r05v_tests.log 2>&1 || { tail -30 gpurun_out/r05v_tests.log; exit 1; }
tail -1 gpurun_out/r05v_tests.log
timeout -k 10 120 ./tools/big_trace_batch.x 256 1024 > gpurun_out/r05v_big_trace_batch.jsonl 2>&1 || { cat gpurun_out/r05v_big_trace_batch.jsonl; exit 1; }
cat gpurun_out/r05v_big_trace_batch.jsonl | cut -c1-260
timeout -k 10 240 python -u tools/big_probe.py > gpurun_out/r05v_big_probe.jsonl 2>&1 || { tail -20 gpurun_out/r05v_big_probe.jsonl; exit 1; }
grep variant gpurun_out/r05v_big_probe.jsonl | cut -c1-150
