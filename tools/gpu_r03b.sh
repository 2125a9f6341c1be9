#!/bin/bash
# R1 / REP identity exit: FastSCL parity files, then FastSCL bench at one and two frame sets.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_schedule_modes.py -q -k "FastSCL or fastscl or golden" --timeout 120 --timeout-method thread > $O/r03b_parity.log 2>&1
rc=$?; tail -4 $O/r03b_parity.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --kind FastSCL-LUT --no-cpu-baseline --no-e2e > $O/r03b_fscl1.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' $O/r03b_fscl1.log
QPD_SETS=2 timeout -k 10 300 python bench.py --kind FastSCL-LUT --no-cpu-baseline --no-e2e > $O/r03b_fscl2.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' $O/r03b_fscl2.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $O/r03b_scl.log 2>&1 || exit $?
grep -o '"value": [0-9.]*' $O/r03b_scl.log
