set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py tests/test_gpu_engine.py -x -q -k "pair_stream or adam_lower" --timeout 200 --timeout-method thread > gpurun_out/r05h_tests.log 2>&1 || { tail -40 gpurun_out/r05h_tests.log; exit 1; }
tail -2 gpurun_out/r05h_tests.log
OUT=gpurun_out/train_r05h
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/ecog -o run -- python3 $GRAFT_REPO_ROOT/tools/train_leg.py ecog 2 > $GRAFT_REPO_ROOT/$OUT/ecog.json 2> $GRAFT_REPO_ROOT/$OUT/ecog.err
cd $GRAFT_REPO_ROOT
python3 tools/train_summary.py $(find $OUT/ecog -name "*kernel_trace.csv") $OUT/ecog.json gpurun_out/r05h_ecog_train_kernels.json | head -16
