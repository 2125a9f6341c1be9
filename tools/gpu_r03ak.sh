#!/bin/bash
# Round 3 ak: interleaved prefix-stage records (coalesced exports / imports, stage 1 off the
# pre-pass row) -- prefix / parity / stream-safety tests, then interleaved A/B against the
# previous commit's build (build_variants/libqpd_prev.so) on the SCL-LUT bench workload.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
show() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$2', round(d['value']/1e6,2), r.get('kernel_ms'), r.get('prefix_kernel_ms'), d['config'].get('prefix_ops'))"; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_prefix.py tests/test_gpu_parity.py tests/test_gpu_stream_safety.py tests/test_gpu_schedule_modes.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03ak_parity.log 2>&1
rc=$?; tail -2 $O/r03ak_parity.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ak_new$r.log 2>&1 || exit $?
show $O/r03ak_new$r.log "SCL-LUT interleaved records"
QPD_LIB=build_variants/libqpd_prev.so timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ak_prev$r.log 2>&1 || exit $?
show $O/r03ak_prev$r.log "SCL-LUT previous (row-major records)"
done
