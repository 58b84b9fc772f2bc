"""Run bench.py's BASELINE configs 1/4/5 section alone (dev tool): python tools/configs_probe.py [--cpu]"""
import json
import os
import sys
import types

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402

args = types.SimpleNamespace(op_seconds=0.6, cpu_seconds=10.0)
dev = torch.device("cuda", 0)
torch.cuda.set_device(0)
stream = torch.cuda.Stream(device=dev)
print(json.dumps(bench.other_configs(args, torch, dev, stream, cpu="--cpu" in sys.argv), indent=1))
