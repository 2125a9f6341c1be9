#!/bin/bash
# Round 3, session a, on the GPU box (repo root): the stream-safety tests, the
# whole GPU suite, smoke, and the SCL-LUT / FastSCL-LUT bench lines.  Stops at
# the first fault / abort / time limit.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
ok01() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }  # pytest: 0 passed, 1 some tests failed
timeout -k 10 300 python -u -m pytest tests/test_gpu_stream_safety.py -v --timeout 120 --timeout-method thread > $O/r03a_stream.log 2>&1
rc=$?; tail -12 $O/r03a_stream.log; ok01 $rc || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r03a_pytest_gpu.log 2>&1
rc=$?; tail -8 $O/r03a_pytest_gpu.log; ok01 $rc || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r03a_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/r03a_bench.log 2>&1 || exit $?
grep '^{' $O/r03a_bench.log
timeout -k 10 300 python bench.py --kind FastSCL-LUT --no-cpu-baseline --no-e2e > $O/r03a_bench_fscl.log 2>&1 || exit $?
grep '^{' $O/r03a_bench_fscl.log
echo "r03a done"
