"""Test configuration: `gpu` marker, import paths for the engine package and the oracle."""
import os
import sys

# torch (the tests' device arithmetic, gloo groups) is imported before the engine library loads: both
# link libamdhip64.so.7, and whichever loads first serves the process.  The other order puts two HIP
# runtimes in one process (the system ROCm's and torch's wheel copy), and torch then sees no GPU
# (tools/torch_hip_probe.py).
import torch  # noqa: F401,E402

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "fhe-sign_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs the HIP path)")
