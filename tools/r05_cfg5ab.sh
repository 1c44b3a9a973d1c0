#!/bin/bash
# cfg5 A/B on the GPU box: old engine vs wave engine on the critical-path
# locus 5949 (alone) and a 2,000-locus batch (bench.py --workload cfg5)
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
for eng in 0 1; do
  WC_WAVE=$eng timeout -k 10 200 python3 -u tools/critical_path.py --top 0 --seeds 5949 --out $O/cp_$eng > $O/cp_$eng.log 2>&1 || exit 1
  head -1 $O/cp_$eng.log
  WC_WAVE=$eng timeout -k 10 400 python3 -u bench.py --workload cfg5 --loci 2000 --steps 1 --warmup 1 --no-cpu > $O/c5_$eng.json 2> $O/c5_$eng.err || exit 1
  python3 -c "import json;d=json.load(open('$O/c5_$eng.json'));print($eng, d['value'], d.get('loci_per_s'), d['kernel_ms_per_step'])"
done
