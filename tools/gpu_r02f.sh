#!/bin/bash
# Round record r02f on the GPU box (repo root): LDS/slab poison diagnosis of the
# fast engine (parity file under build_variants/libqpd_poison*.so), then the
# GPU suite, smoke, the SCL-LUT and FastSCL-LUT bench lines and a rocprofv3
# kernel-stats pass.  Stops at the first fault / abort / time limit.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
ok01() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }  # pytest: 0 passed, 1 some tests failed
for v in ${POISON:-poisonF poison0}; do
  if [ -f build_variants/libqpd_$v.so ]; then
    QPD_LIB=build_variants/libqpd_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q \
      --timeout 120 --timeout-method thread > $O/r02f_$v.log 2>&1
    rc=$?; tail -15 $O/r02f_$v.log; ok01 $rc || exit $rc
  fi
done
timeout -k 10 400 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r02f_pytest_gpu.log 2>&1
rc=$?; tail -8 $O/r02f_pytest_gpu.log; ok01 $rc || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $O/r02f_smoke.log 2>&1 || exit $?
timeout -k 10 300 python bench.py > $O/r02f_bench.log 2>&1 || exit $?
grep '^{' $O/r02f_bench.log
timeout -k 10 300 python bench.py --kind FastSCL-LUT --no-cpu-baseline > $O/r02f_bench_fscl.log 2>&1 || exit $?
grep '^{' $O/r02f_bench_fscl.log
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r02f_kt_fscl -o kt --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --kind FastSCL-LUT > $O/r02f_kt_fscl.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r02f_kt_scl -o kt --output-format csv -- \
  python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e > $O/r02f_kt_scl.log 2>&1 || exit $?
echo "r02f done"
