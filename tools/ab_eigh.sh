set -o pipefail
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_eigh.py tests/test_gpu_diag_gf.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t_eigh.log 2>&1 || { tail -30 gpurun_out/t_eigh.log; exit 1; }
tail -2 gpurun_out/t_eigh.log
for g in 512 1024 2048; do echo "grid $g fused" ; ED_GPU_TRLAN_GRID=$g timeout -k 10 120 python tools/eigh_prof.py 2>&1 | grep eigh | tail -1 || exit 1; done
echo "unfused 512"; ED_GPU_TRLAN_UNFUSED=1 ED_GPU_TRLAN_GRID=512 timeout -k 10 120 python tools/eigh_prof.py 2>&1 | grep eigh | tail -1
