#!/bin/bash
# Round 3 i: generator deposit by 16-bit halves (product) and the generator's
# occupancy (launch-bounds variants mc6 / mc8), end-to-end rate and mc kernel time.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_montecarlo.py -m gpu -q --timeout 120 --timeout-method thread > $O/r03i_pytest_mc.log 2>&1
rc=$?; tail -3 $O/r03i_pytest_mc.log; [ $rc -eq 0 ] || exit $rc
: > $O/r03i_ab.txt
for round in 1 2; do
  for lib in prod mc6 mc8; do
    if [ $lib = prod ]; then unset QPD_LIB; else export QPD_LIB=build_variants/libqpd_$lib.so; fi
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 4 > $O/r03i_tmp.log 2>&1 || exit $?
    grep '^{' $O/r03i_tmp.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); e=r['monte_carlo_e2e']; print('$round $lib', round(r['value']/1e6,2), round(e['value']/1e6,2), round(e['mc_kernel_ms'],3))" | tee -a $O/r03i_ab.txt
  done
done
unset QPD_LIB
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY -d $O/r03i_pmc_mc -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $O/r03i_pmc_mc.log 2>&1 || echo "pmc pass failed"
echo done
