#!/bin/bash
# Round 3 aa: FastSCL R1 argsort rounds run lazily per layer (product) vs the
# previous commit (prev): parity tests, then an interleaved A/B.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_schedule_modes.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03aa_pytest.log 2>&1
rc=$?; tail -3 $O/r03aa_pytest.log; [ $rc -eq 0 ] || exit $rc
: > $O/r03aa_ab.txt
for round in 1 2; do
  for lib in prev prod; do
    if [ $lib = prod ]; then unset QPD_LIB; else export QPD_LIB=build_variants/libqpd_$lib.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 4 --kind FastSCL-LUT > $O/r03aa_tmp.log 2>&1 || exit $?
    echo "$round $lib FastSCL-LUT $(grep -o '"value": [0-9.]*' $O/r03aa_tmp.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $O/r03aa_tmp.log)" | tee -a $O/r03aa_ab.txt
  done
done
echo done
