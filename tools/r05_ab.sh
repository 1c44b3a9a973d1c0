#!/bin/bash
# one_sub.py A/B on the GPU box: old engine vs wave engine, timing + phase profile
# bash tools/r05_ab.sh <tag> <seed> [workload]
export TMPDIR=/tmp
T=$1; SEED=$2; WL=${3:-cfg5-hpc}
O=gpurun_out/$T
mkdir -p $O
WC_WAVE=0 timeout -k 10 120 python3 tools/one_sub.py --workload $WL --seed $SEED > $O/old.json || exit 1
WC_WAVE=1 timeout -k 10 120 python3 tools/one_sub.py --workload $WL --seed $SEED > $O/wave.json || exit 1
WC_WAVE=1 WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 120 python3 tools/one_sub.py --workload $WL --seed $SEED --phases /tmp/ph.txt > $O/wave_ph.json || exit 1
cat $O/old.json $O/wave.json $O/wave_ph.json
