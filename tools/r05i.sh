set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_primitives.py -x -v -k "potrf" --timeout 200 --timeout-method thread > gpurun_out/r05i_tests.log 2>&1 || { tail -40 gpurun_out/r05i_tests.log; exit 1; }
tail -3 gpurun_out/r05i_tests.log
timeout -k 10 120 python tools/potrf_ab.py 4096 2048 > gpurun_out/r05i_potrf_ab.json 2> gpurun_out/r05i_potrf_ab.err || { tail -20 gpurun_out/r05i_potrf_ab.err; exit 1; }
cat gpurun_out/r05i_potrf_ab.json
OUT=gpurun_out/stress_r05i
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$OUT/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/potrf_timeline.py > $GRAFT_REPO_ROOT/$OUT/trace.log 2>&1
cd $GRAFT_REPO_ROOT
python3 tools/potrf_timeline.py --show $(find $OUT/trace -name "*kernel_trace.csv") > gpurun_out/r05i_stress_potrf_timeline.txt
head -12 gpurun_out/r05i_stress_potrf_timeline.txt; tail -1 gpurun_out/r05i_stress_potrf_timeline.txt
