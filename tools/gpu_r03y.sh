#!/bin/bash
# Round 3 y: current-build bench lines for the other configurations and kinds:
# BASELINE config 2 (SC-LUT N=128 K=32, MinDistortion Q=16), SC-LUT / FastSC-LUT
# N=1024, CA-SCL-LUT / CA-FastSCL-LUT N=1024 L=8.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
: > $O/r03y_kinds.jsonl
for spec in "SC-LUT 128 32 1" "SC-LUT 1024 512 1" "FastSC-LUT 1024 512 1" "CA-SCL-LUT 1024 512 8" "CA-FastSCL-LUT 1024 512 8"; do
  set -- $spec
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --kind $1 --N $2 --K $3 --L $4 > $O/r03y_tmp.log 2>&1 || exit $?
  grep '^{' $O/r03y_tmp.log >> $O/r03y_kinds.jsonl
  tail -1 $O/r03y_kinds.jsonl | python -c "import json,sys; r=json.loads(sys.stdin.read()); print('$1', $2, $3, $4, round(r['value']/1e6,2), 'M frames/s', round(r['roofline']['kernel_ms'],3), 'ms', r['ber'], r['bler'])"
done
echo done
