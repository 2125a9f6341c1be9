#!/bin/bash
# Round 3 am: sanity check of the committed tree's library -- smoke, prefix tests, one bench line.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r03am_smoke.log 2>&1 || exit $?
tail -1 $O/r03am_smoke.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_prefix.py tests/test_gpu_stream_safety.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03am_prefix.log 2>&1
rc=$?; tail -1 $O/r03am_prefix.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/r03am_bench.log 2>&1 || exit $?
grep '^{' $O/r03am_bench.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', round(d['value']/1e6,2), d['roofline']['kernel_ms'], d['roofline']['prefix_kernel_ms'])"
