#!/bin/bash
# Round 3 z: frame sets per wave (QPD_SETS 1 vs the default 2) for the
# single-path kinds SC-LUT / FastSC-LUT at N = 1024 and SC-LUT at N = 128.
set -u
cd "$GRAFT_REPO_ROOT"
O=gpurun_out
mkdir -p $O
: > $O/r03z_sets.txt
for round in 1 2; do
  for spec in "SC-LUT 1024 512" "FastSC-LUT 1024 512" "SC-LUT 128 32"; do
    set -- $spec
    for sets in 2 1; do
      QPD_SETS=$sets timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --steps 4 --kind $1 --N $2 --K $3 --L 1 > $O/r03z_tmp.log 2>&1 || exit $?
      echo "$round sets=$sets $1 $2 $(grep -o '"value": [0-9.]*' $O/r03z_tmp.log | head -1) $(grep -o '"kernel_ms": [0-9.]*' $O/r03z_tmp.log)" | tee -a $O/r03z_sets.txt
    done
  done
done
echo done
