#!/bin/bash
# Round 3 an: CA-SCL-LUT bench line on the frozen-prefix build (the CRC-aided kind takes the same stages).
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python bench.py --kind CA-SCL-LUT --no-cpu-baseline --no-e2e > $O/r03an_ca_scl.log 2>&1 || exit $?
grep '^{' $O/r03an_ca_scl.log > $O/r03an_ca_scl.jsonl
python -c "import json; d=json.loads(open('$O/r03an_ca_scl.jsonl').read()); print('CA-SCL-LUT', round(d['value']/1e6,2), d['roofline']['kernel_ms'], d['roofline']['prefix_kernel_ms'], d['config']['prefix_ops'])"
