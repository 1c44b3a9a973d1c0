#!/bin/bash
# GPU box: wave kernels at 1 vs 2 waves per SIMD (alone: 5949 / 1525 full
# level), and the 2000-locus cfg5 batch: priority for predicted-slow loci on
# and off, and the 1-wave build
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
W1=$PWD/waffle_con_amd/libwaffle_con_w1.so
for seed in 5949 1525; do
  timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed $seed > $O/s${seed}.log 2>&1 || exit 1
  WAFFLE_CON_LIB=$W1 timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed $seed > $O/s${seed}_w1.log 2>&1 || exit 1
  echo $seed $(grep -o '"us_per_pop": [0-9.]*' $O/s${seed}.log) w1 $(grep -o '"us_per_pop": [0-9.]*' $O/s${seed}_w1.log)
done
for v in prio noprio w1; do
  case $v in
    prio) E="WC_PRIO_FRAC=0.02";; noprio) E="WC_PRIO_FRAC=0";; w1) E="WAFFLE_CON_LIB=$W1";;
  esac
  env $E timeout -k 10 300 python3 -u tools/cfg5_lat.py --loci 2000 --out $O/lat_$v > $O/lat_$v.log 2>&1 || { tail -20 $O/lat_$v.log; exit 1; }
  echo $v; grep -v amdgpu.ids $O/lat_$v.log | head -4
done
