#!/bin/bash
# GPU box: tools/votes_diag.py on the given library variants
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
for v in "$@"; do
  echo "== $v"
  WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_$v.so timeout -k 10 300 python3 -u tools/votes_diag.py > $O/vd_$v.log 2>&1 || { tail -5 $O/vd_$v.log; exit 1; }
  grep -v amdgpu $O/vd_$v.log | tail -8
done
