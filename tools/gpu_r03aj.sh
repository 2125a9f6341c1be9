#!/bin/bash
# Round 3 aj: frozen-prefix stages at two frame sets per wave (QPD_PFX_SETS=2, the new default)
# vs one -- prefix / parity tests, then two interleaved A/B rounds on the SCL-LUT bench workload.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
show() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$2', round(d['value']/1e6,2), r.get('kernel_ms'), r.get('prefix_kernel_ms'), d['config'].get('prefix_ops'))"; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_prefix.py tests/test_gpu_parity.py tests/test_gpu_stream_safety.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03aj_parity.log 2>&1
rc=$?; tail -2 $O/r03aj_parity.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03aj_sets2_$r.log 2>&1 || exit $?
show $O/r03aj_sets2_$r.log "SCL-LUT prefix sets=2"
QPD_PFX_SETS=1 timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03aj_sets1_$r.log 2>&1 || exit $?
show $O/r03aj_sets1_$r.log "SCL-LUT prefix sets=1"
done
