#!/bin/bash
# Host engine behind the C-ABI: its GPU tests, the whole GPU suite, then the
# per-frame latency tool (host engine, one-frame GPU call, the reference).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_host_engine.py -q --timeout 120 --timeout-method thread > $O/r03d_host_engine.log 2>&1
rc=$?; tail -5 $O/r03d_host_engine.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 500 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r03d_pytest_gpu.log 2>&1
rc=$?; tail -5 $O/r03d_pytest_gpu.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python tools/latency.py 300 > $O/r03d_latency.jsonl 2> $O/r03d_latency.err || exit $?
cat $O/r03d_latency.jsonl
