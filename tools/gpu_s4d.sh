#!/bin/bash
# -m gpu suite + full bench line at HEAD
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s4d}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
timeout -k 10 500 python3 bench.py > "$OUT/bench.log" 2>&1 || { tail -30 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" > "$OUT/bench.json"
python3 -c "import json,sys; d=json.load(open('$OUT/bench.json')); print(d['value'], json.dumps(d['batched_c2']))"
