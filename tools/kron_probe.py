"""bench.py's kron_mv leg alone, three times (python tools/kron_probe.py): us per call and GB/s."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
for _ in range(3):
    r = bench.kron_mv_leg(dev)
    print(json.dumps({k: r[k] for k in ("us_per_call", "achieved_GBs", "frac", "check_rel_err")}))
