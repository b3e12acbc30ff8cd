#!/bin/bash
# (diagnostics) per-workgroup timestamps of the band-state pass under A/B environments
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 2
for v in ${STAMP_VARIANTS:-"HZ_AB_CHAIN=0" "HZ_AB_CHAIN=4" "HZ_AB_CHAIN=7"}; do
  echo "== $v"
  env ${v//,/ } HZ_AB_STAMPS=1 timeout -k 10 120 python bench.py --steps 20 --warmup 2 --no-cpu-baseline --no-traffic \
      --no-per-sample --side-steps 0 --stream-blocks 0 2>&1 | grep stamps
done
