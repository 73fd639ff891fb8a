set -eo pipefail
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/s4a
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_nccl.py -x -v --timeout 240 --timeout-method thread > gpurun_out/s4a/nccl.log 2>&1 || { tail -40 gpurun_out/s4a/nccl.log; exit 1; }
tail -3 gpurun_out/s4a/nccl.log
timeout -k 10 400 python -u tools/farm_scale_probe.py --out gpurun_out/s4a/farm_scale.json > gpurun_out/s4a/farm_scale.log 2>&1
tail -8 gpurun_out/s4a/farm_scale.log
