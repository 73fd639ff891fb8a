set -o pipefail
for r in 1 2; do
 for v in base loc2 ru; do
  ED_LIB=ab/libedgpu_$v.so timeout -k 10 100 python -u tools/eigh_prof.py 6 6 2>&1 | grep eigh | tail -2 | sed "s/^/$v /" || exit 1
  ED_LIB=ab/libedgpu_$v.so timeout -k 10 100 python -u tools/eigh_prof.py 3 4 2>&1 | grep eigh | tail -1 | sed "s/^/$v /" || exit 1
 done
done
for r in 1 2; do
 for v in base loc2 ru; do
  timeout -k 10 100 python -u tools/farm_prof.py --reps 3 --batch-max-dim 0 --lib ab/libedgpu_$v.so 2>&1 | grep wall | sed "s/^/$v /" || exit 1
 done
done
