#!/bin/bash
# Round 3 p: right specials / leaves run their parent's combine (MF_PCOMB):
# GPU suite, then A/B against QPD_NO_PCOMB=1 (the same build without the fusion).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03p_pytest_gpu.log 2>&1
rc=$?; tail -3 $O/r03p_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
: > $O/r03p_ab.txt
for round in 1 2; do
  for kind in FastSCL-LUT SCL-LUT FastSC-LUT; do
    for v in off on; do
      if [ $v = off ]; then export QPD_NO_PCOMB=1; else unset QPD_NO_PCOMB; fi
      timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 4 --kind $kind > $O/r03p_tmp.log 2>&1 || exit $?
      echo "$round pcomb=$v $kind $(grep -o '"value": [0-9.]*' $O/r03p_tmp.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $O/r03p_tmp.log) $(grep -o '"ops": [0-9]*' $O/r03p_tmp.log)" | tee -a $O/r03p_ab.txt
    done
  done
done
echo done
