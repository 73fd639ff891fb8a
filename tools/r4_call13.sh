#!/bin/bash
# Round 4, call 13: MODE 4 slot-major LDS vector with absolute addressing
# (no per-gather address adds): parity, then the configs[1] rates.
set -o pipefail
export RUN=${RUN:-r4o}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
bash tools/gpu_step.sh \
 "tests:500:python -u -m pytest tests/test_gpu_lanczos.py tests/test_gpu_diag_gf.py tests/test_gpu_golden.py tests/test_gpu_kron_split.py tests/test_bench_launch.py tests/test_gpu_nccl.py -x -q -m gpu --timeout 500 --timeout-method thread" \
 "bench:300:python bench.py --no-farm --no-roofline --no-cpu > $O/bench_c2.json" \
 "cvec:120:python3 $R/tools/cvec_probe.py"
du -sh $O
