#!/bin/bash
# Round 3 v: machine-scheduler strategy max-memory-clause for the SCL unit
# (s_mmc) and for the FastSCL unit (f_mmc) against the product build.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
: > $O/r03v_ab.txt
for round in 1 2; do
  for pair in "SCL-LUT s_mmc" "FastSCL-LUT f_mmc"; do
    set -- $pair
    for lib in prod $2; do
      if [ $lib = prod ]; then unset QPD_LIB; else export QPD_LIB=build_variants/libqpd_$lib.so; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 4 --kind $1 > $O/r03v_tmp.log 2>&1 || exit $?
      echo "$round $lib $1 $(grep -o '"value": [0-9.]*' $O/r03v_tmp.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $O/r03v_tmp.log)" | tee -a $O/r03v_ab.txt
    done
  done
done
echo done
