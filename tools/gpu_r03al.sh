#!/bin/bash
# Round 3 al: final records of the round's build -- GPU suite, smoke, the default bench line
# (with the reference CPU baseline and the Monte-Carlo rate), the 10^8-frame point, then
# rocprofv3 kernel statistics + PMC passes of the SCL-LUT bench workload.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > $O/r03al_pytest_gpu.log 2>&1
rc=$?; tail -2 $O/r03al_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/r03al_smoke.log 2>&1 || exit $?
tail -1 $O/r03al_smoke.log
timeout -k 10 400 python bench.py > $O/r03al_bench.log 2>&1 || exit $?
grep '^{' $O/r03al_bench.log > $O/r03al_bench.jsonl
timeout -k 10 300 python bench.py --mc-frames 1e8 > $O/r03al_mc_1e8.log 2>&1 || exit $?
grep '^{' $O/r03al_mc_1e8.log > $O/r03al_mc_1e8.jsonl
echo "records done"
timeout -k 10 600 bash tools/profile_round.sh r03al_scl --kind SCL-LUT > $O/r03al_prof_scl.log 2>&1 || exit $?
echo "profile done"
