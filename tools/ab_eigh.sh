# A/B of the device thick-restart eigh (run on the GPU box from the repo root)
set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_eigh.py tests/test_gpu_diag_gf.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_eigh.log 2>&1 || { tail -30 gpurun_out/t_eigh.log; exit 1; }
tail -2 gpurun_out/t_eigh.log
for g in ${GRIDS:-512}; do echo "grid $g fused" ; ED_GPU_TRLAN_GRID=$g timeout -k 10 120 python tools/eigh_prof.py 2>&1 | grep eigh | tail -1 || exit 1; done
