#!/bin/bash
# GPU box: the cfg2 e2e leg with 16 / 12 / 8 / 4 staging threads
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for t in 16 12 8 4; do
  WC_UPLOAD_THREADS=$t timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu --cfg5-loci 0 > $O/e2e_$t.json 2> $O/e2e_$t.err || { tail -20 $O/e2e_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/e2e_$t.json'));print($t, round(d['e2e_loci_per_s']), round(d['e2e_upload_ms'],1), round(d['e2e_compute_ms'],1), round(d['loci_per_s']))"
done
