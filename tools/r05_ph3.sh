#!/bin/bash
# GPU box: cfg3 locus 0 alone (normal and phase builds) and cfg5 5949 / 1525 full-read level
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg3 --seed 0 > $O/s0.log 2>&1 || exit 1
grep us_per_pop $O/s0.log
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg3 --seed 0 --phases /tmp/ph_c3.txt > $O/ph_c3.log 2>&1 || exit 1
grep -v amdgpu $O/ph_c3.log | tail -1
for seed in 5949 1525; do
  timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed $seed > $O/s$seed.log 2>&1 || exit 1
  grep us_per_pop $O/s$seed.log
done
