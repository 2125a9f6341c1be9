#!/bin/bash
# Round 3 ad: frozen-prefix split as a PFX template argument of lut_fast_kernel
# (no wrapper) -- GPU suite, then interleaved A/B against the HEAD build.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
show() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$2', round(d['value']/1e6,2), r.get('kernel_ms'), r.get('prefix_kernel_ms'), d['config'].get('prefix_ops'))"; }
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03ad_pytest_gpu.log 2>&1
rc=$?; tail -2 $O/r03ad_pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for k in SCL-LUT FastSCL-LUT; do
    timeout -k 10 300 python bench.py --kind $k --no-cpu-baseline --no-e2e > $O/r03ad_${k}_new$r.log 2>&1 || exit $?
    show $O/r03ad_${k}_new$r.log "$k new"
    QPD_LIB=build_variants/libqpd_head.so timeout -k 10 300 python bench.py --kind $k --no-cpu-baseline --no-e2e > $O/r03ad_${k}_head$r.log 2>&1 || exit $?
    show $O/r03ad_${k}_head$r.log "$k head"
  done
done
