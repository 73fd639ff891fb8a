# farm A/B over (workers, small_workers[, cache_budget_mb]), alternating
# configurations, 3 runs x 4 reps each:
#   bash tools/farm_sw.sh OUTNAME "8 6" "8 0" "8 6 256" ...
O=gpurun_out/$1; shift
mkdir -p $O
CFGS=("$@")
for i in 1 2 3; do for c in "${CFGS[@]}"; do read -r w s b <<< "$c"
  echo "== workers $w small_workers $s budget ${b:-default}" >> $O/sw.log
  timeout -k 10 150 python tools/farm_prof.py --reps 4 --workers $w --small-workers $s ${b:+--budget $b} >> $O/sw.log 2>&1 || exit 1
done; done
