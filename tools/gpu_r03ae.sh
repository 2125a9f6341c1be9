#!/bin/bash
# Round 3 ae: two frozen-prefix stages for SCL-LUT (stage 2: <= 4 live paths at L = 4)
# -- prefix tests + parity files, then interleaved A/B: two stages / stage 1 only
# (QPD_NO_PFX2=1) / the HEAD build.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
show() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$2', round(d['value']/1e6,2), r.get('kernel_ms'), r.get('prefix_kernel_ms'), d['config'].get('prefix_ops'))"; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_prefix.py tests/test_gpu_parity.py tests/test_gpu_schedule_modes.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03ae_parity.log 2>&1
rc=$?; tail -2 $O/r03ae_parity.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ae_two$r.log 2>&1 || exit $?
  show $O/r03ae_two$r.log "SCL-LUT two-stage"
  QPD_NO_PFX2=1 timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ae_one$r.log 2>&1 || exit $?
  show $O/r03ae_one$r.log "SCL-LUT stage-1"
  QPD_LIB=build_variants/libqpd_head.so timeout -k 10 300 python bench.py --kind SCL-LUT --no-cpu-baseline --no-e2e > $O/r03ae_head$r.log 2>&1 || exit $?
  show $O/r03ae_head$r.log "SCL-LUT head"
done
