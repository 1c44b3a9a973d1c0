#!/bin/bash
# PMC views of one cfg5-hpc sub-problem alone (tools/one_sub.py), old vs wave engine:
#   bash tools/pmc_wave.sh <tag> <seed> "<counters>"
export TMPDIR=/tmp
T=$1; SEED=$2; C=$3
O=gpurun_out/$T
mkdir -p $O
for eng in 0 1; do
  WC_WAVE=$eng timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $O/pmc_$eng -o run -- python3 tools/one_sub.py --seed $SEED > $O/pmc_$eng.json || exit 1
done
echo done
