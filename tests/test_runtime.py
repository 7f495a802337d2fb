"""One HIP runtime per process.  Root cause of the old "many contexts -> torch.cuda
hipErrorNoDevice" report: PyTorch-ROCm bundles its own libamdhip64.so / libhsa-runtime64.so, loaded
by file name from torch/lib, while libshs_gpu.so binds the system ROCm runtime by SONAME.  With the
library loaded first, the process mapped two HIP + HSA runtimes and torch's device enumeration failed
-- with one context as with 64 (tools/diag_runtime.py on the MI355X box).  shs_gpu._abi.load() now
loads torch's runtime first when torch is installed, so both share it.  Each case runs in a fresh
child process; this process never initialises the GPU for them."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r'''
import ctypes, json, sys
sys.path.insert(0, "leisure-software-renderer_amd")
n = int(sys.argv[1])
from shs_gpu import _abi
lib = _abi.load()                          # before any torch import
out = {}
if n:
    hs = []
    for i in range(n):
        h = ctypes.c_void_p()
        assert lib.shs_create(0, ctypes.byref(h)) == 0, i
        hs.append(h)
    for h in hs:
        lib.shs_destroy(h)
    import torch
    torch.cuda.init()
    out["torch_sum"] = float(torch.ones(4, device="cuda").sum().item())
maps = open("/proc/self/maps").read().split("\n")
out["hip"] = sorted({l.split()[-1] for l in maps if "libamdhip64" in l and "/" in l})
out["hsa"] = sorted({l.split()[-1] for l in maps if "libhsa-runtime64" in l and "/" in l})
print(json.dumps(out))
'''


def _run(n):
    r = subprocess.run([sys.executable, "-c", CHILD, str(n)], cwd=ROOT, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_library_maps_one_hip_runtime():
    """Loading libshs_gpu.so maps exactly one HIP and one HSA runtime (torch's when torch is installed)."""
    out = _run(0)
    assert len(out["hip"]) == 1 and len(out["hsa"]) == 1, out
    try:
        import importlib.util
        has_torch = importlib.util.find_spec("torch") is not None
    except ImportError:
        has_torch = False
    if has_torch:
        assert "torch" in out["hip"][0], out


@pytest.mark.gpu
def test_many_contexts_then_torch_cuda():
    """64 shs contexts created and destroyed, then torch.cuda initialised, in that order."""
    out = _run(64)
    assert out["torch_sum"] == 4.0
    assert len(out["hip"]) == 1 and len(out["hsa"]) == 1, out
