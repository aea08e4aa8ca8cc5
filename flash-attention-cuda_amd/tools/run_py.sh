#!/bin/bash
# run one tools/*.py on the box with a time limit, output to gpurun_out/<name>.jsonl
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}/flash-attention-cuda_amd" || exit 1
mkdir -p ../gpurun_out
name=$1; shift
timeout -k 10 ${TLIM:-300} python tools/$name.py "$@" > ../gpurun_out/$name.jsonl 2>&1
