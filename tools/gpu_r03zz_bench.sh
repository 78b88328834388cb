#!/bin/bash
# Final default bench line with the r03zz profile set in the tree (roofline.profile cites it).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out
timeout -k 10 400 python -u bench.py > gpurun_out/r03zz_bench_final.json 2> gpurun_out/r03zz_bench_final.err || { tail -20 gpurun_out/r03zz_bench_final.err; exit 1; }
python -c "
import json;d=json.loads(open('gpurun_out/r03zz_bench_final.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['profile'], d['roofline']['avg_launch_us'], d['roofline']['frac'])"
