#!/bin/bash
# Round 4, call 7: parity of the k_direct / CGS changes, k_direct times,
# farm A/B (local-only update vs full), complex MODE 4 LDS counters, the
# k_direct setup profile (k_gen_diag), and last the 8-worker profiled farm
# that crashed in round 3, with the process's shared-object map for
# symbolising (core dumps off).
set -o pipefail
export RUN=${RUN:-r4g}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py"
F="python3 $R/tools/farm_prof.py"
bash tools/gpu_step.sh \
 "tests:500:python -u -m pytest tests/test_gpu_hxv.py tests/test_gpu_jz.py tests/test_gpu_dist.py tests/test_gpu_golden.py tests/test_gpu_eigh.py tests/test_gpu_lanczos.py tests/test_gpu_diag_gf.py -x -q --timeout 200 --timeout-method thread" \
 "probe:180:$P --sector n26s --path 1 --iters 30 && $P --sector n28 --path 1 --iters 30 && $P --sector n28j --path 1 --iters 30 && $P --sector n26s --path 1 --iters 30 --cvec" \
 "farm_def:180:$F --reps 3" \
 "farm_fullupd:180:$F --reps 3 --options trlan_fullupd" \
 "serial_def:240:$F --reps 1 --serial-stats $O/serial_def.json" \
 "cvec:120:python3 $R/tools/cvec_probe.py" \
 "pmc_cvec:120:bash tools/pmc_pass.sh $O pmc_cvec 'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU' python3 $R/tools/cvec_probe.py" \
 "st_direct:150:cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $O/st_direct_n28 -o st --output-format csv -- python3 $R/tools/spmv_probe.py --sector n28 --path 1 --iters 30" \
 "crash:200:ulimit -c 0; cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $O/fp_w8ng -o fp --output-format csv -- python3 $R/tools/farm_prof.py --workers 8 --reps 1 --options no_graph --maps $O/maps_w8ng.json"
