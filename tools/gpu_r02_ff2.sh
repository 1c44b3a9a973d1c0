set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_ff2
mkdir -p $O
for v in 0 2; do
  WC_NARROW=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > $O/cfg2_n$v.json 2> $O/cfg2_n$v.err || { echo "cfg2 n$v failed"; tail $O/cfg2_n$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg2_n$v.json')); print('narrow=$v cfg2 loci/s', round(d['loci_per_s']), 'kernel ms', round(d['kernel_ms_per_step'],2), 'step ms', round(d['ms_per_step'],2))"
done
