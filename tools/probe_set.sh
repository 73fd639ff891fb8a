#!/bin/bash
# H·v timing of the stored / matrix-free kernels on the SURVEY §8(d) sweep
# sectors (tools/spmv_probe.py per line); usage: tools/probe_set.sh [set]
set -o pipefail
case "${1:-all}" in
  direct) L=("--sector n28 --path 1" "--sector n28 --path 1 --cvec" "--sector n28b --path 1"
             "--sector n28j --path 1" "--sector n26s --path 1" "--sector c4 --path 1" "--sector c2 --path 1") ;;
  stored) L=("--sector n28 --path 0" "--sector n28 --path 0 --complex" "--sector n28b --path 0"
             "--sector n28j --path 0" "--sector n28j --path 0 --complex" "--sector n26s --path 0"
             "--sector n26s --path 0 --complex") ;;
  *) L=("--sector n28 --path 0" "--sector n28 --path 1" "--sector n28 --path 2" "--sector n28 --path 1 --cvec"
        "--sector n28b --path 1" "--sector n28j --path 0" "--sector n28j --path 1" "--sector n26s --path 0"
        "--sector n26s --path 1" "--sector c4 --path 1" "--sector c2 --path 1") ;;
esac
for a in "${L[@]}"; do
  python tools/spmv_probe.py $a --iters ${ITERS:-30} 2>&1 | grep -v amdgpu.ids || exit 1
done
