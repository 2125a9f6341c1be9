# Round-6 record, part 2 (GPU box, repo root): rocprofv3 kernel stats + PMC passes of the
# SCL-LUT and FastSCL-LUT bench workloads (-> profiles/counters.json), config C5's 10^8-frame
# point, the L = 16 line (lane groups of 16) and config C2.
cd "$GRAFT_REPO_ROOT"
TAG=r06zg
step() { local name=$1; shift; "$@" > gpurun_out/${TAG}_$name.log 2>&1; local rc=$?; echo "[$name rc=$rc]"; grep -v amdgpu.ids gpurun_out/${TAG}_$name.log | tail -2 | cut -c1-300; [ $rc -eq 0 ] || exit $rc; }
step prof_scl bash tools/profile_round.sh ${TAG}_scl --kind SCL-LUT
step prof_fscl bash tools/profile_round.sh ${TAG}_fscl --kind FastSCL-LUT
step mc timeout -k 10 300 python bench.py --mc-frames 1e8 --no-cpu-baseline
step bench_l16 timeout -k 10 300 python bench.py --L 16 --frames 1048576 --no-e2e
step bench_c2 timeout -k 10 300 python bench.py --kind SC-LUT --N 128 --K 32 --frames 16777216 --no-e2e
