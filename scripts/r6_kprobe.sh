#!/bin/bash
# (probe) kernel-argument read latency against a device buffer (scripts/probe/kernarg_probe.hip)
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
mkdir -p gpurun_out/r6
/opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 -Wno-unused-result scripts/probe/kernarg_probe.hip -o gpurun_out/r6/kernarg_probe 2>/dev/null || exit 1
timeout -k 10 60 gpurun_out/r6/kernarg_probe && HIP_FORCE_DEV_KERNARG=0 timeout -k 10 60 gpurun_out/r6/kernarg_probe
