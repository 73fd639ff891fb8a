#!/bin/bash
# full -m gpu suite at HEAD, c4 (6,6) one-pass vs forced two-pass matrix-free,
# then the roofline sweep (kernel stats + PMC passes) and the bench line
set -eo pipefail
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${1:-s4c}
mkdir -p "$OUT"
cd "$R"
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > "$OUT/gpu_tests.log" 2>&1 || { tail -30 "$OUT/gpu_tests.log"; exit 1; }
tail -2 "$OUT/gpu_tests.log"
for k in 0 1; do
  ED_GPU_KRON2=$k timeout -k 10 120 python3 tools/spmv_probe.py --sector c4r --path 2 --iters 50 | tee -a "$OUT/c4_kron.log"
done
bash tools/gpu_sweep.sh "${1:-s4c}_sweep"
