#!/bin/bash
# GPU box: cfg2 phase profile (300 loci) with the phase build
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 400 python3 -u tools/phase_run.py --workload cfg2 --loci 300 --out $O/ph > $O/ph.log 2>&1 || { tail -20 $O/ph.log; exit 1; }
python3 -c "import json;d=json.load(open('$O/ph/report.json'));print(json.dumps({k:d[k] for k in d if k in ('kernel_ms','pops','phase_share')}))"
