#!/bin/bash
# Same-box A/B between a previous tree and the current one, interleaved.
# usage (GPU box, repo root): bash tools/ab_tree.sh <prev_dir> <tag> [rounds] [train]
#   <prev_dir>  a copy of the previous commit with its library built in place (e.g. a git worktree under the repo,
#               git-excluded, which gpurun's snapshot carries to the box)
#   rounds      PM2.5 bench runs per tree (300 graph-replayed steps each, the other legs off)
#   train       "train": also one HCP (20 steps) and one ECoG (2 steps) graph_train leg per tree
# Output: gpurun_out/<tag>_ab.txt, one line per run: <tree> <round> <it/s> <ms/step> <final loss>
#         and for the training legs: <leg> <tree> <s/step> <loss>
R=${GRAFT_REPO_ROOT:-$(pwd)}
PREV=$1; TAG=$2; ROUNDS=${3:-3}; TRAIN=${4:-}
cd "$R" || exit 1
mkdir -p gpurun_out
OUT=gpurun_out/${TAG}_ab.txt
: > $OUT
leg() {  # leg <tree> <dir> <round>
  local name=$1 dir=$2 r=$3
  local j="$R/gpurun_out/${TAG}_${name}_${r}.json"
  (cd "$dir" && timeout -k 10 300 python -u bench.py --no-breakdown --no-cpu-baseline --no-stress --no-elbo \
      --no-api --no-hcp --no-ecog --no-kron --steps 300 --warmup 30 > "$j" 2> "${j%.json}.err") || return 1
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); \
print(sys.argv[2], sys.argv[3], d['value'], d['ms_per_step'], d.get('final_loss'))" "$j" "$name" "$r" >> $OUT
}
for r in $(seq 1 $ROUNDS); do
  leg prev "$PREV" $r || { echo "prev run $r failed"; tail -5 gpurun_out/${TAG}_prev_${r}.err; exit 1; }
  leg new . $r || { echo "new run $r failed"; tail -5 gpurun_out/${TAG}_new_${r}.err; exit 1; }
done
if [ "$TRAIN" = train ]; then
  for cfg in hcp ecog; do
    for t in prev new; do
      dir=$PREV; [ $t = new ] && dir=.
      (cd "$dir" && timeout -k 10 400 python -u -c "
import sys, torch, bench
torch.cuda.set_device(0)
d = bench.graph_train(torch.device('cuda', 0), '$cfg', steps=20 if '$cfg' == 'hcp' else 2, warmup=1)
print('$cfg', '$t', d['s_per_step'], d['loss'])" >> "$R/$OUT" 2> "$R/gpurun_out/${TAG}_${t}_${cfg}.err") \
        || { echo "$cfg $t failed"; tail -5 gpurun_out/${TAG}_${t}_${cfg}.err; exit 1; }
    done
  done
fi
cat $OUT
