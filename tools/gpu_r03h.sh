#!/bin/bash
# Round 3 h: generator parity (new log / sincos / quantizer walk), the bench
# line with the fused end-to-end rate, and the LDS-budget trade-off of the
# SCL-LUT kernel (frames/s and HBM-side bytes per frame vs the depths kept in LDS).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_montecarlo.py tests/test_gpu_stream_safety.py -m gpu -q --timeout 120 --timeout-method thread > $O/r03h_pytest_mc.log 2>&1
rc=$?; tail -3 $O/r03h_pytest_mc.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/r03h_bench.log 2>&1 || exit $?
grep '^{' $O/r03h_bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); e=r['monte_carlo_e2e']; print(r['value'], r['roofline']['kernel_ms'], e['value'], e['mc_kernel_ms'])"
: > $O/r03h_lds.txt
for b in 10240 14336 20480 30720; do
  QPD_LDS_BUDGET=$b timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 3 > $O/r03h_tmp.log 2>&1 || exit $?
  echo "budget $b $(grep -o '"value": [0-9.]*' $O/r03h_tmp.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $O/r03h_tmp.log) $(grep -o '"lds_from_depth": [0-9]*' $O/r03h_tmp.log)" | tee -a $O/r03h_lds.txt
done
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for b in 10240 20480; do
  for c in FETCH_SIZE WRITE_SIZE; do
    QPD_LDS_BUDGET=$b timeout -s KILL 120 rocprofv3 --pmc $c -d $O/r03h_pmc_${b}_$c -o p --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e > $O/r03h_pmc_${b}_$c.log 2>&1 || exit $?
  done
done
echo done
