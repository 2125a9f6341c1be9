#!/bin/bash
# Round 3 z2: FastSC-LUT on one frame set by default: GPU parity suite + bench line.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r03z2_pytest_gpu.log 2>&1
rc=$?; tail -3 $O/r03z2_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --kind FastSC-LUT > $O/r03z2_tmp.log 2>&1 || exit $?
grep '^{' $O/r03z2_tmp.log > $O/r03z2_fastsc.jsonl
grep -o '"value": [0-9.]*' $O/r03z2_fastsc.jsonl | head -1
