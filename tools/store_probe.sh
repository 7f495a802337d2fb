#!/bin/bash
# Build tools/libstore_probe.so (tools/store_probe.hip) for gfx950; timing tool for tools/store_rate.py.
cd "$(dirname "$0")" && /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -shared -o libstore_probe.so store_probe.hip
