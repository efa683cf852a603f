"""The bench's parity-mode line alone (NerfRunner.train() batches: N_rand=2048 over the
64-frame pool, graph replay), for a kernel-trace profile of the small-batch step."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402

dev = torch.device("cuda", 0)
e, _ = bench.side_line({}, 64, 2048, dev, 20, int(os.environ.get("STEPS", "50")), parity=True,
                       graph=os.environ.get("GRAPH", "1") == "1")
print(json.dumps(e))
