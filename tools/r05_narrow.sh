#!/bin/bash
# GPU box: cfg2 with the single engine's 128-thread build (WC_NARROW=3) vs default (2)
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for rep in 1 2; do
  for nm in 2 3; do
    WC_NARROW=$nm timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --no-e2e --cfg5-loci 0 > $O/n${nm}_$rep.json 2> $O/n${nm}_$rep.err || { tail -20 $O/n${nm}_$rep.err; exit 1; }
    python3 -c "import json;d=json.load(open('$O/n${nm}_$rep.json'));print('WC_NARROW=$nm', $rep, round(d['loci_per_s']), round(d['ms_per_step'],2), round(d['roofline']['kernel_ms_per_launch'],2))"
  done
done
