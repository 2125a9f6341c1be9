# Round 6 j (GPU box, repo root): per-op-class stamps of the round's kernels (diagnostic
# build build_variants/libqpd_stamps.so: -DQPD_STAMPS) for SCL-LUT, FastSCL-LUT and SCL-LUT at
# L = 16; the SCL-LUT batch-size sweep; the other kinds on the bench workload.
cd "$GRAFT_REPO_ROOT"
set -o pipefail
for a in "SCL-LUT 1024 512 8 262144" "FastSCL-LUT 1024 512 8 262144" "SCL-LUT 1024 512 16 131072"; do
  QPD_LIB=build_variants/libqpd_stamps.so timeout -k 10 120 python tools/stamps.py $a 2>&1 | grep -v amdgpu.ids || exit 1
done > gpurun_out/r06j_stamps.txt
for f in 65536 262144 1048576 2097152; do
  timeout -k 10 200 python bench.py --frames $f --steps 5 --warmup 1 --no-cpu-baseline --no-e2e 2>/dev/null | tail -1 || exit 1
done > gpurun_out/r06j_batch.jsonl
AB_TAG=tree timeout -k 10 300 python tools/ab_kinds.py CA-SCL-LUT CA-FastSCL-LUT SC-LUT FastSC-LUT CA-SCL-LUT:16 2>&1 \
  | grep -v amdgpu.ids > gpurun_out/r06j_kinds.txt || exit 1
cat gpurun_out/r06j_stamps.txt gpurun_out/r06j_kinds.txt
python -c "
import json
for l in open('gpurun_out/r06j_batch.jsonl'):
    d = json.loads(l); print(d['config']['frames_per_gpu_per_step'], round(d['value'] / 1e6, 2))"
