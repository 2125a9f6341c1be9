set -u
cd "$GRAFT_REPO_ROOT"
: > gpurun_out/ab3.txt
for v in fgi3 comb fgi3 comb; do QPD_LIB=build_variants/libqpd_$v.so AB_TAG=$v timeout -k 10 150 python tools/ab_kinds.py SCL-LUT FastSCL-LUT >> gpurun_out/ab3.txt 2>&1 || exit $?; done
grep -v amdgpu.ids gpurun_out/ab3.txt
