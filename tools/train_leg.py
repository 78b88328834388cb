"""One of bench.py's fp32 training legs alone (GPU box), for rocprofv3 kernel traces of the HCP / ECoG steps:
python tools/train_leg.py {hcp|ecog} [steps].  Prints bench.graph_train's JSON (setup, warm-up and the timed
graph replays; the trace summary divides by the replays it sees)."""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

cfg = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else (10 if cfg == "hcp" else 2)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
print(json.dumps(bench.graph_train(dev, cfg, steps=steps, warmup=1)), flush=True)
