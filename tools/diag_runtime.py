"""Diagnose the 'many contexts -> torch.cuda hipErrorNoDevice' report: each case runs
in a fresh child process (this parent never touches the GPU) and prints which HIP / HSA runtime files
the process has mapped and whether torch.cuda comes up after N shs contexts."""
import json
import subprocess
import sys

CHILD = r'''
import ctypes, json, sys
sys.path.insert(0, "leisure-software-renderer_amd")
n, order = int(sys.argv[1]), sys.argv[2]
out = {"n_contexts": n, "order": order}
if order == "torch_first":
    import torch
from shs_gpu import _abi
lib = _abi.load()
hs = []
for i in range(n):
    h = ctypes.c_void_p()
    rc = lib.shs_create(0, ctypes.byref(h))
    if rc:
        out["create_failed_at"] = i
        break
    hs.append(h)
for h in hs:
    lib.shs_destroy(h)
import torch
try:
    torch.cuda.init()
    out["torch_cuda"] = "ok"
    out["torch_device_count"] = torch.cuda.device_count()
    x = torch.ones(4, device="cuda")
    out["torch_sum"] = float(x.sum().item())
except Exception as e:
    out["torch_cuda"] = repr(e)[:200]
maps = open("/proc/self/maps").read().split("\n")
libs = sorted({l.split()[-1] for l in maps if ("libamdhip64" in l or "libhsa-runtime64" in l) and "/" in l})
out["runtime_files"] = libs
print(json.dumps(out))
'''


def main():
    cases = [(1, "shs_first"), (64, "shs_first"), (64, "torch_first")]
    for n, order in cases:
        r = subprocess.run([sys.executable, "-c", CHILD, str(n), order], capture_output=True, text=True, timeout=300)
        line = [l for l in r.stdout.splitlines() if l.startswith("{")]
        print(line[-1] if line else json.dumps({"n": n, "order": order, "rc": r.returncode, "stderr": r.stderr[-400:]}))
        sys.stdout.flush()


if __name__ == "__main__":
    main()
