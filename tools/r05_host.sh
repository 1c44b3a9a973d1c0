#!/bin/bash
# GPU box: cfg2 bench steps with the library's host timing lines
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
WC_HOST_TIMING=1 timeout -k 10 300 python3 -u bench.py --steps 5 --warmup 1 --no-cpu --no-e2e --cfg5-loci 0 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
grep "\[wc\]" $O/b.err | tail -12
python3 -c "import json;d=json.load(open('$O/b.json'));print(d['value'], d['ms_per_step'], d['roofline']['kernel_ms_per_launch'])"
