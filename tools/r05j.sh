set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 120 python tools/potrf_ab.py 4096 2048 > gpurun_out/r05j_potrf_ab.json 2> gpurun_out/r05j_potrf_ab.err || { tail -20 gpurun_out/r05j_potrf_ab.err; exit 1; }
cat gpurun_out/r05j_potrf_ab.json
