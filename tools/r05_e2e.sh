#!/bin/bash
# GPU box: the cfg2 e2e leg with 16 / 12 / 8 staging threads
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
for t in 16 12 8; do
  WC_UPLOAD_THREADS=$t timeout -k 10 300 python3 -u bench.py --no-cpu --cfg5-loci 0 --steps 10 --warmup 3 > $O/e2e_$t.json 2> $O/e2e_$t.err || { tail -5 $O/e2e_$t.err; exit 1; }
  python3 -c "import json;d=json.load(open('$O/e2e_$t.json'));print('threads $t', d['value'], d.get('e2e_loci_per_s'), d.get('e2e_upload_ms'), d.get('e2e_compute_ms'))"
done
