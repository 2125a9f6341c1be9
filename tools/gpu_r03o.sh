#!/bin/bash
# Round 3 o: BER/BLER curves 0-5 dB (driver's stop rule) for SCL-LUT and
# FastSCL-LUT, each point's first frames checked bit-exact against the reference.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
timeout -k 10 400 python tools/ber_sweep.py --kind SCL-LUT > $O/r03o_ber_scl.jsonl 2> $O/r03o_ber_scl.err || exit $?
timeout -k 10 400 python tools/ber_sweep.py --kind FastSCL-LUT > $O/r03o_ber_fscl.jsonl 2> $O/r03o_ber_fscl.err || exit $?
cat $O/r03o_ber_scl.jsonl $O/r03o_ber_fscl.jsonl | cut -c1-330
