set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u bench.py > gpurun_out/r05a_bench.json 2> gpurun_out/r05a_bench.err
tail -1 gpurun_out/r05a_bench.json | cut -c1-400
bash tools/syrk_inside_pmc.sh
python3 - <<'P'
import json
for k in ("stress","ecog"):
    d=json.load(open(f"gpurun_out/syrkin/{k}_mfma.json"))
    print(k, len(d["rows"]))
P
