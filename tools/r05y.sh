set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
bash tools/train_pmc.sh r05zz
cp gpurun_out/r05zz_hcp_train_traffic.json gpurun_out/r05zz_ecog_train_traffic.json profiles/
timeout -k 10 600 python -u bench.py > gpurun_out/r05zz_bench2.json 2> gpurun_out/r05zz_bench2.err || { tail -20 gpurun_out/r05zz_bench2.err; exit 1; }
python3 -c "
import json; d=json.loads(open('gpurun_out/r05zz_bench2.json').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'])
for k in ('hcp_train','ecog_train'):
  r=d[k]['roofline']; print(k, d[k]['s_per_step'], r['kernel'][:30], r.get('traffic'), r.get('traffic_GBs_over_busy_time'), r.get('traffic_stale'))
"
