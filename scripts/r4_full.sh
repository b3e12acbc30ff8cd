# the whole GPU suite (one process), as the driver runs it
set -o pipefail
mkdir -p gpurun_out/r4
timeout -k 10 1500 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r4/pytest_full.log 2>&1; echo "pytest rc=$?" >> gpurun_out/r4/pytest_full.log
