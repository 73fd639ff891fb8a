#!/bin/bash
# A/B of library builds on the thick-restart path: the lone (6,6) and (3,4)
# configs[3] solves (tools/eigh_prof.py) and the 8-worker farm without the
# small-sector batch (tools/farm_prof.py), alternating builds, two rounds.
#   bash tools/ab_cgs.sh NAME=path/to/libedgpu.so [NAME=...]
set -o pipefail
for r in 1 2; do
  for kv in "$@"; do
    v=${kv%%=*}; lib=${kv#*=}
    ED_LIB=$lib timeout -k 10 100 python -u tools/eigh_prof.py 6 6 2>&1 | grep eigh | tail -2 | sed "s/^/$v /" || exit 1
    ED_LIB=$lib timeout -k 10 100 python -u tools/eigh_prof.py 3 4 2>&1 | grep eigh | tail -1 | sed "s/^/$v /" || exit 1
  done
done
for r in 1 2; do
  for kv in "$@"; do
    v=${kv%%=*}; lib=${kv#*=}
    timeout -k 10 100 python -u tools/farm_prof.py --reps 3 --batch-max-dim 0 --lib "$lib" 2>&1 | grep wall | sed "s/^/$v /" || exit 1
  done
done
