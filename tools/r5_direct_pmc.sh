#!/bin/bash
# k_direct on the nonSU2 N26 sector: the counter passes of tools/pmc_passes.txt
# (one pass per line, each under its own limit), then the 8-worker farm under
# rocprofv3 (graphs off).  Output in gpurun_out/r5pmc.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$R" || exit 2
O=$R/gpurun_out/r5pmc
mkdir -p "$O"
n=0
while read -r ctr; do
  [ -z "$ctr" ] && continue
  n=$((n + 1))
  bash tools/pmc_pass.sh "$O" "direct_n26s_p$n" "$ctr" python3 "$R/tools/spmv_probe.py" --sector n26s --path 1 --iters 5 \
    || exit 1
done < tools/pmc_passes.txt
RUN=r5pmc bash tools/split_ab.sh "d26s:-:--sector n26s --path 1" "d26s_pf:tools/variants/lib_dirpf.so:--sector n26s --path 1" \
  "d28_pf:tools/variants/lib_dirpf.so:--sector n28 --path 1" "d28:-:--sector n28 --path 1" || exit 1
RUN=r5pmc bash tools/farm_rocprof.sh w8nograph || exit 1
echo PMC_DONE
