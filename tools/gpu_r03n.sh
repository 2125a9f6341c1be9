#!/bin/bash
# Round 3 n: generator noise pairs per lane and round / waves per SIMD
# (prod = 2 pairs at 6 waves; p4w5, p4w6, p1w6): mc kernel time and e2e rate.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
: > $O/r03n_ab.txt
for round in 1 2; do
  for lib in prod p4w5 p4w6 p1w6; do
    if [ $lib = prod ]; then unset QPD_LIB; else export QPD_LIB=build_variants/libqpd_$lib.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 3 > $O/r03n_tmp.log 2>&1 || exit $?
    grep '^{' $O/r03n_tmp.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); e=r['monte_carlo_e2e']; print('$round $lib', round(r['value']/1e6,3), round(e['value']/1e6,3), round(e['mc_kernel_ms'],3))" | tee -a $O/r03n_ab.txt
  done
done
echo done
