# Round-6 record, part 1 (GPU box, repo root): the GPU suite, smoke(), the SCL-LUT and FastSCL-LUT bench lines.
cd "$GRAFT_REPO_ROOT"
TAG=r06zg
mkdir -p gpurun_out
step() { local name=$1; shift; "$@" > gpurun_out/${TAG}_$name.log 2>&1; local rc=$?; echo "[$name rc=$rc]"; grep -v amdgpu.ids gpurun_out/${TAG}_$name.log | tail -2 | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step pytest timeout -k 10 540 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
step smoke timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()"
step bench timeout -k 10 300 python bench.py
step bench_fscl timeout -k 10 300 python bench.py --kind FastSCL-LUT
