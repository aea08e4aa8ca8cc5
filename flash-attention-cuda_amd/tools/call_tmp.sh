#!/bin/bash
# run-to-run spread of the bench line on one box (three back-to-back processes)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --no-sweep --no-cpu-baseline --no-pmc 2>/dev/null | tail -1 || exit 1
done > gpurun_out/bench_repeat.jsonl
python - <<'PY'
import json
for l in open("gpurun_out/bench_repeat.jsonl"):
    d = json.loads(l); print(d["value"], d["ms_per_step"])
PY
