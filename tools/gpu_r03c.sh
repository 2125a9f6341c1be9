#!/bin/bash
# Per-op-class wave cycles (stamps build) for FastSCL-LUT at one / two frame sets and SCL-LUT.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
export QPD_LIB=build_variants/libqpd_stamps.so STAMPS_DEPTH=1
timeout -k 10 200 python tools/stamps.py FastSCL-LUT 1024 512 8 262144 > $O/r03c_stamps_fscl1.txt 2>&1 || exit $?
QPD_SETS=2 timeout -k 10 200 python tools/stamps.py FastSCL-LUT 1024 512 8 262144 > $O/r03c_stamps_fscl2.txt 2>&1 || exit $?
timeout -k 10 200 python tools/stamps.py SCL-LUT 1024 512 8 262144 > $O/r03c_stamps_scl.txt 2>&1 || exit $?
head -3 $O/r03c_stamps_*.txt
