#!/bin/bash
# Build and run tools/graph_edge_repro2.hip's patterns (one process each: a segfault ends only its pattern).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out tools/bin
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/graph_edge_repro2.hip -o tools/bin/graph_edge_repro2 || exit 1
for p in base mfirst s2k nojoin2 s1only; do
  timeout -k 5 60 tools/bin/graph_edge_repro2 $p > gpurun_out/graph_repro2_$p.log 2>&1
  echo "$p rc=$? $(tr '\n' ' ' < gpurun_out/graph_repro2_$p.log)"
done
# the same binary on the HIP runtime torch bundles (ROCm 7.0; the Python process's runtime) instead of /opt/rocm's 7.2
TL=$(python -c "import torch,os;print(os.path.join(os.path.dirname(torch.__file__),'lib'))")
mkdir -p /tmp/tlib && ln -sf $TL/libamdhip64.so /tmp/tlib/libamdhip64.so.7
for p in base s2k; do
  LD_LIBRARY_PATH=/tmp/tlib:$TL timeout -k 5 60 tools/bin/graph_edge_repro2 $p > gpurun_out/graph_repro2_torchrt_$p.log 2>&1
  echo "torch-runtime $p rc=$? $(tr '\n' ' ' < gpurun_out/graph_repro2_torchrt_$p.log)"
done
