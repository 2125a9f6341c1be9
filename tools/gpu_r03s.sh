#!/bin/bash
# Round 3 s: generator Horner steps as v_fma_f64 with SGPR constants (product) vs the previous commit (prev).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_montecarlo.py -m gpu -q --timeout 120 --timeout-method thread > $O/r03s_pytest_mc.log 2>&1
rc=$?; tail -3 $O/r03s_pytest_mc.log; [ $rc -eq 0 ] || exit $rc
: > $O/r03s_ab.txt
for round in 1 2 3; do
  for lib in prev prod; do
    if [ $lib = prod ]; then unset QPD_LIB; else export QPD_LIB=build_variants/libqpd_$lib.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 > $O/r03s_tmp.log 2>&1 || exit $?
    grep '^{' $O/r03s_tmp.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); e=r['monte_carlo_e2e']; print('$round $lib', round(r['value']/1e6,3), round(e['value']/1e6,3), round(e['ms_per_step'],3), round(e['mc_kernel_ms'],3))" | tee -a $O/r03s_ab.txt
  done
done
echo done
