#!/bin/bash
# Round-3 pass U: one graphed PM2.5 step's kernel timeline of the current code.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r03u_trace -o run -- python3 $R/bench.py --steps 30 --warmup 5 --no-breakdown --no-cpu-baseline --no-stress --no-elbo --no-api --no-hcp --no-ecog > $R/gpurun_out/r03u_trace.json 2> $R/gpurun_out/r03u_trace.err || exit $?
cd $R
python tools/step_timeline.py $(find gpurun_out/r03u_trace -name "*kernel_trace.csv") > gpurun_out/r03u_timeline.txt
cat gpurun_out/r03u_timeline.txt
