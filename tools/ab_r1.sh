set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu_r1.log 2>&1 || { tail -30 gpurun_out/pytest_gpu_r1.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_r1.log
export SWEEP_FRAMES=262144 SWEEP_WAVES=0
SWEEP_BUDGETS=6144,8192 timeout -k 10 240 python tools/sweep.py FastSCL-LUT 1024 512 8 2>&1 | grep -v amdgpu.ids
QPD_SETS=2 SWEEP_BUDGETS=10240,12288 timeout -k 10 240 python tools/sweep.py FastSCL-LUT 1024 512 8 2>&1 | grep -v amdgpu.ids
SWEEP_BUDGETS=10240 timeout -k 10 240 python tools/sweep.py SCL-LUT 1024 512 8 2>&1 | grep -v amdgpu.ids
SWEEP_BUDGETS=10240 timeout -k 10 240 python tools/sweep.py CA-FastSCL-LUT 1024 512 8 2>&1 | grep -v amdgpu.ids
