# farm A/B: small_workers 0 vs 6 (8 workers), alternating runs, 4 reps each
mkdir -p gpurun_out/r6sw3
for i in 1 2 3 4 5; do for sw in 0 6; do
  echo "== small_workers $sw" >> gpurun_out/r6sw3/sw.log
  timeout -k 10 150 python tools/farm_prof.py --reps 4 --small-workers $sw >> gpurun_out/r6sw3/sw.log 2>&1 || exit 1
done; done
