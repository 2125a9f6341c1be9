#!/bin/bash
# Round 3 f: GPU suite (host engine NaN flag, fused Monte-Carlo test), per-frame
# latency, the SCL bench line with the fused end-to-end rate, then the
# non-inlined special-op A/B for FastSCL-LUT (tools/gpu_r03e.sh).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r03f_pytest_gpu.log 2>&1
rc=$?; tail -5 $O/r03f_pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/latency.py 300 > $O/r03f_latency.jsonl 2> $O/r03f_latency.err || exit $?
cat $O/r03f_latency.jsonl
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/r03f_bench.log 2>&1 || exit $?
grep '^{' $O/r03f_bench.log | python -c "import json,sys; r=json.loads(sys.stdin.read()); print(r['value'], r['monte_carlo_e2e'])"
bash tools/gpu_r03e.sh
