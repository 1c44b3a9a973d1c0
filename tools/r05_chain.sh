#!/bin/bash
# GPU box: the full-read level of cfg5 locus 5949 alone on the dual builds:
# block engine, block engine with dual chains (WC_DUAL_CHAIN=k), wave engine
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
run() {  # tag env...
  local tag=$1; shift
  env "$@" timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed 5949 > $O/$tag.log 2>&1 || { tail -5 $O/$tag.log; return 1; }
  echo $tag $(grep us_per_pop $O/$tag.log)
}
run block WC_WAVE=0 && run chain16 WC_WAVE=0 WC_DUAL_CHAIN=16 && run chain32 WC_WAVE=0 WC_DUAL_CHAIN=32 && run wave WC_WAVE=1 && \
WC_WAVE=0 WC_DUAL_CHAIN=16 WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed 5949 --phases /tmp/ph_c.txt > $O/chain16_ph.log 2>&1 && grep -v amdgpu $O/chain16_ph.log
