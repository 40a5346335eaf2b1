"""Probe: does torch see the GPU when the engine (system ROCm HIP runtime) initialised HIP first, and in
the reverse order?  usage: python3 tools/torch_hip_probe.py engine-first|torch-first"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fhe-sign_amd"))
order = sys.argv[1]
print({k: v for k, v in os.environ.items() if "VISIBLE" in k or k.startswith(("HIP", "HSA", "ROCR", "GPU"))})
if order == "torch-first":
    import torch
    print("torch first:", torch.cuda.is_available(), torch.cuda.device_count())
from fhe_sign import Context  # noqa: E402
ctx = Context(0)
print("engine context ok")
import torch  # noqa: E402
print(order, "torch:", torch.cuda.is_available(), torch.cuda.device_count())
maps = [l.split()[-1] for l in open("/proc/self/maps") if "amdhip64" in l or "hsa-runtime" in l]
print(sorted(set(maps)))
ctx.close()
