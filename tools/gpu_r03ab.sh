#!/bin/bash
# Round 3 ab: frozen-prefix split (lut_prefix_kernel) -- parity files, then the
# bench workload with and without the split (QPD_NO_PFX=1), SCL-LUT and FastSCL-LUT.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
show() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$2', round(d['value']/1e6,2), r.get('kernel_ms'), r.get('prefix_kernel_ms'), d['config'].get('prefix_ops'))"; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_prefix.py tests/test_gpu_parity.py tests/test_gpu_schedule_modes.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03ab_parity.log 2>&1
rc=$?; tail -3 $O/r03ab_parity.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for k in SCL-LUT FastSCL-LUT; do
    timeout -k 10 300 python bench.py --kind $k --no-cpu-baseline --no-e2e > $O/r03ab_${k}_pfx$r.log 2>&1 || exit $?
    show $O/r03ab_${k}_pfx$r.log "$k pfx"
    QPD_NO_PFX=1 timeout -k 10 300 python bench.py --kind $k --no-cpu-baseline --no-e2e > $O/r03ab_${k}_nopfx$r.log 2>&1 || exit $?
    show $O/r03ab_${k}_nopfx$r.log "$k nopfx"
  done
done
