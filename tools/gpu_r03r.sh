#!/bin/bash
# Round-3 pass R: where torch's capture of the side<->side2 ping-pong crashes (host-side segfault in a child):
# keep_graph capture (EndCapture alone, then a dot dump, then instantiate), and the raw HIP sequence on
# streams created with priorities like torch's stream pool.  Child processes; the GPU is not faulted.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
PROBE_KEEP_GRAPH=1 PROBE_OUT_CHARS=4000 timeout -k 10 120 python -u tools/graph_edge_probe.py fork_join ping_pong > gpurun_out/r03r_graph_keep.jsonl 2>&1
cat gpurun_out/r03r_graph_keep.jsonl
for v in "prio=0" "prio=-1"; do
  timeout -k 10 60 ./tools/bin/graph_edge_repro ping_pong global autofree $v > gpurun_out/r03r_graph_prio.txt 2>&1
  rcg=$?; echo "hip ping_pong [$v] rc=$rcg: $(tr '\n' ' ' < gpurun_out/r03r_graph_prio.txt)"
  [ $rcg -ne 0 ] && break
done
exit 0
