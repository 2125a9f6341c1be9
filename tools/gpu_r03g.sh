#!/bin/bash
# Round 3 g: GPU suite on the product build (pipelined shallow ops, generator
# grid / error counting), the bench line with the fused end-to-end rate, then an
# interleaved A/B against the round's committed HEAD (build_variants/libqpd_head.so).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r03g_pytest_gpu.log 2>&1
rc=$?; tail -5 $O/r03g_pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/r03g_bench.log 2>&1 || exit $?
grep '^{' $O/r03g_bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['roofline']['kernel_ms'], r['monte_carlo_e2e'])"
: > $O/r03g_ab.txt
for round in 1 2; do
  for kind in SCL-LUT FastSCL-LUT; do
    for lib in head prod; do
      if [ $lib = head ]; then export QPD_LIB=build_variants/libqpd_head.so; else unset QPD_LIB; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 4 --kind $kind > $O/r03g_tmp.log 2>&1 || exit $?
      echo "$round $lib $kind $(grep -o '"value": [0-9.]*' $O/r03g_tmp.log) $(grep -o '"kernel_ms": [0-9.]*' $O/r03g_tmp.log)" | tee -a $O/r03g_ab.txt
    done
  done
done
