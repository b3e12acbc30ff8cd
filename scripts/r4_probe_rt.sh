set -o pipefail
mkdir -p gpurun_out/r4
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 120 python -u scripts/probe/rt_beside.py 256 > gpurun_out/r4/rt_beside.log 2>&1 && \
timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/r4/rt_beside_trace -o t --output-format csv -- \
  python3 scripts/probe/rt_beside.py 256 >> gpurun_out/r4/rt_beside.log 2>&1
