#!/bin/bash
# Two-rank gloo rehearsal of the HCP-shaped data-parallel step on a one-GPU box (both ranks on cuda:0):
# flat and bucketed all-reduce timings, then one bucketed run with rank 0 under a rocprofv3 kernel + memory-copy
# trace (no counters), whose timeline shows where the communication stream's copies start relative to the gradient
# graph's last kernels.  -> gpurun_out/<tag>_hcp_n2_{flat,bucketed}.json, gpurun_out/<tag>_hcp_n2_bucketed_trace.txt
TAG=${1:-r06}
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 1
mkdir -p gpurun_out
export MASTER_ADDR=127.0.0.1 WORLD_SIZE=2
pair() {   # pair <port> <mode> <steps> <out> [profile dir]
  local port=$1 mode=$2 steps=$3 out=$R/$4 prof=$5
  export MASTER_PORT=$port
  RANK=1 LOCAL_RANK=1 timeout -k 10 500 python3 tools/dp_hcp_rehearsal.py $mode $steps > /dev/null 2> $out.r1.err &
  local p1=$!
  if [ -n "$prof" ]; then
    (cd /tmp && export TMPDIR=/tmp && RANK=0 LOCAL_RANK=0 timeout -k 10 500 rocprofv3 --kernel-trace \
      --memory-copy-trace --output-format csv -d $prof -o run -- python3 $R/tools/dp_hcp_rehearsal.py $mode $steps \
      > $out 2> $out.r0.err)
  else
    RANK=0 LOCAL_RANK=0 timeout -k 10 500 python3 tools/dp_hcp_rehearsal.py $mode $steps > $out 2> $out.r0.err
  fi
  local rc=$?
  wait $p1
  local rc1=$?
  [ $rc -ne 0 ] && { echo "rank 0 failed rc=$rc"; tail -5 $out.r0.err; return 1; }
  [ $rc1 -ne 0 ] && { echo "rank 1 failed rc=$rc1"; tail -5 $out.r1.err; return 1; }
  tail -1 $out
}
if [ -z "$PROFILE_ONLY" ]; then
  pair 29611 flat 3 gpurun_out/${TAG}_hcp_n2_flat.json || exit 1
  pair 29612 bucketed 3 gpurun_out/${TAG}_hcp_n2_bucketed.json || exit 1
fi
pair 29613 bucketed 2 gpurun_out/${TAG}_hcp_n2_bucketed_prof.json $R/gpurun_out/dp_$TAG || exit 1
python3 tools/dp_trace_summary.py $(find gpurun_out/dp_$TAG -name "*kernel_trace.csv" | head -1) \
  $(find gpurun_out/dp_$TAG -name "*memory_copy_trace.csv" | head -1) > gpurun_out/${TAG}_hcp_n2_bucketed_trace.txt
cat gpurun_out/${TAG}_hcp_n2_bucketed_trace.txt | head -30
