#!/bin/bash
# Round 3 ac: frozen-prefix split restricted to SCL-LUT, metric resumed by an
# import op -- prefix tests + parity file, then interleaved A/B against the
# HEAD build (build_variants/libqpd_head.so) on the bench workload.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
show() { grep '^{' "$1" | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d.get('roofline',{}); print('$2', round(d['value']/1e6,2), r.get('kernel_ms'), r.get('prefix_kernel_ms'), d['config'].get('prefix_ops'))"; }
timeout -k 10 500 python -u -m pytest tests/test_gpu_prefix.py tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/r03ac_parity.log 2>&1
rc=$?; tail -2 $O/r03ac_parity.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for k in SCL-LUT FastSCL-LUT; do
    timeout -k 10 300 python bench.py --kind $k --no-cpu-baseline --no-e2e > $O/r03ac_${k}_new$r.log 2>&1 || exit $?
    show $O/r03ac_${k}_new$r.log "$k new"
    QPD_LIB=build_variants/libqpd_head.so timeout -k 10 300 python bench.py --kind $k --no-cpu-baseline --no-e2e > $O/r03ac_${k}_head$r.log 2>&1 || exit $?
    show $O/r03ac_${k}_head$r.log "$k head"
  done
done
