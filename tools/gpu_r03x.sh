#!/bin/bash
# Round 3 x: __builtin_expect on the identity fast path of the leaf forks (product) vs the previous commit (prev).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03x_pytest_gpu.log 2>&1
rc=$?; tail -3 $O/r03x_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
: > $O/r03x_ab.txt
for round in 1 2; do
  for kind in SCL-LUT FastSCL-LUT; do
    for lib in prev prod; do
      if [ $lib = prod ]; then unset QPD_LIB; else export QPD_LIB=build_variants/libqpd_$lib.so; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 4 --kind $kind > $O/r03x_tmp.log 2>&1 || exit $?
      echo "$round $lib $kind $(grep -o '"value": [0-9.]*' $O/r03x_tmp.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $O/r03x_tmp.log)" | tee -a $O/r03x_ab.txt
    done
  done
done
echo done
