#!/bin/bash
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 300 python3 -u tools/step_split.py 1000 > $O/split.log 2>&1 || { tail -20 $O/split.log; exit 1; }
grep step $O/split.log
