#!/bin/bash
# HBM fetch of the static persistent order vs the dynamic-queue experiment build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
export TMPDIR=/tmp
O=../gpurun_out/dynq_fetch
mkdir -p $O
for v in base dynq; do
  for shp in "64 32 4096" "1 32 8192"; do
    set -- $shp
    timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $O/${v}_$1_$3 -o f --output-format csv -- python tools/lib_fetch.py $v $1 $2 $3 4 > $O/${v}_$1_$3.log 2>&1 || exit 1
  done
done
