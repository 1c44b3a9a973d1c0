#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python3 -u tools/cfg4_path.py --out $O > $O/c4p.log 2>&1 || { tail -20 $O/c4p.log; exit 1; }
grep -v amdgpu $O/c4p.log
