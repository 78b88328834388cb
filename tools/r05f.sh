set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_engine.py tests/test_gpu_ecog.py -x -v -s -k "pair_stream or ragged or ecog or adam_lower" --timeout 300 --timeout-method thread > gpurun_out/r05f_tests.log 2>&1 || { grep -E "PARITY|PAIR_STREAM|PASS|FAIL|Error|error" gpurun_out/r05f_tests.log | tail -40; tail -30 gpurun_out/r05f_tests.log; exit 1; }
grep -E "PARITY|PAIR_STREAM|passed|failed" gpurun_out/r05f_tests.log | tail -30
timeout -k 10 600 python -u tools/train_leg.py ecog 2 > gpurun_out/r05f_ecog.json 2> gpurun_out/r05f_ecog.err || { tail -20 gpurun_out/r05f_ecog.err; exit 1; }
tail -1 gpurun_out/r05f_ecog.json | cut -c1-600
