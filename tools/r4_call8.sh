#!/bin/bash
# Round 4, call 8: parity of the probe screen / coefficient-column changes,
# k_direct times, complex MODE 4 LDS counters, the k_direct setup profile,
# eigensolver and farm A/B (probe screen, local-only update, 128-block
# sweeps), and the 8-worker profiled farm with its shared-object map; large
# traces deleted (the copy-back limit is 64 MiB).
set -o pipefail
export RUN=${RUN:-r4h}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/$RUN
P="python3 $R/tools/spmv_probe.py"
F="python3 $R/tools/farm_prof.py"
bash tools/gpu_step.sh \
 "tests:500:python -u -m pytest tests/test_gpu_eigh.py tests/test_gpu_golden.py tests/test_gpu_lanczos.py tests/test_gpu_diag_gf.py tests/test_gpu_hxv.py -x -q --timeout 200 --timeout-method thread" \
 "trlan_ab:300:python3 $R/tools/trlan_ab.py --reps 3 --opts eigh_fullprobe,trlan_fullupd,eigh_no_verify,trlan_g128" \
 "farm_def:180:$F --reps 3" \
 "farm_fullprobe:180:$F --reps 3 --options eigh_fullprobe" \
 "farm_g128:180:$F --reps 3 --options trlan_g128" \
 "probe:180:$P --sector n26s --path 1 --iters 30 && $P --sector n28 --path 1 --iters 30 && $P --sector n28j --path 1 --iters 30 && $P --sector n26s --path 1 --iters 30 --cvec" \
 "pmc_cvec:120:bash tools/pmc_pass.sh $O pmc_cvec 'SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_INSTS_SALU' python3 $R/tools/cvec_probe.py" \
 "st_direct:150:cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $O/st_direct_n28 -o st --output-format csv -- python3 $R/tools/spmv_probe.py --sector n28 --path 1 --iters 30 && find $O/st_direct_n28 -name '*kernel_trace.csv' -size +2M -delete" \
 "crash:200:ulimit -c 0; cd /tmp && export TMPDIR=/tmp && rocprofv3 --kernel-trace --stats -d $O/fp_w8ng -o fp --output-format csv -- python3 $R/tools/farm_prof.py --workers 8 --reps 1 --options no_graph --maps $O/maps_w8ng.json; rc=\$?; find $O/fp_w8ng -name '*kernel_trace.csv' -delete; exit \$rc"
du -sh $O
