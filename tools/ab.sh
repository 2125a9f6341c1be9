set -e
cd $GRAFT_REPO_ROOT
export SWEEP_BUDGETS=${SWEEP_BUDGETS:-5120,6144} SWEEP_FRAMES=262144 SWEEP_WAVES=0
for v in $VARIANTS; do
  echo "== $v"
  QPD_LIB=build_variants/libqpd_$v.so timeout -k 10 240 python tools/sweep.py SCL-LUT 1024 512 8
done
