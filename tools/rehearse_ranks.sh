#!/bin/bash
# Rehearsal of bench.py's N-rank path on a one-GPU box: `--gpus 2` self-launches
# two ranks (torch.distributed.run) that share cuda:0 and reduce over gloo.
# The Monte-Carlo point must give the same counters at 1 and 2 ranks (frames
# keyed by global frame id).  usage (GPU box, repo root): bash tools/rehearse_ranks.sh
set -eu
cd "$GRAFT_REPO_ROOT"
export QPD_BENCH_DEVICES=0 QPD_BENCH_BACKEND=gloo
timeout -k 10 300 python bench.py --gpus 2 --no-cpu-baseline --steps 3 > gpurun_out/rehearse_bench2.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --mc-frames 4e6 --frames 131072 > gpurun_out/rehearse_mc1.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --mc-frames 4e6 --frames 131072 > gpurun_out/rehearse_mc2.log 2>&1
timeout -k 10 300 python bench.py --gpus 2 --mc-frames 4e6 --frames 131072 --mc-stop 1000 > gpurun_out/rehearse_mc2s.log 2>&1
timeout -k 10 300 python bench.py --gpus 1 --mc-frames 4e6 --frames 131072 --mc-stop 1000 > gpurun_out/rehearse_mc1s.log 2>&1
for f in bench2 mc1 mc2 mc1s mc2s; do grep "^{" gpurun_out/rehearse_$f.log | python3 -c "
import json, sys
d = json.loads(sys.stdin.read())
print('$f', d['n_gpus'], round(d['value'] / 1e6, 2), {k: d.get(k) for k in ('ber', 'bler', 'bit_errors', 'block_errors', 'blocks', 'frames_counted')})"; done
