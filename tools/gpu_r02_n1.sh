# narrow (128-thread) engine build: parity suite, cfg2 A/B, cfg5 A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_n1
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
for v in 1 0; do
  WC_NARROW=$v timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > $O/cfg2_n$v.json 2> $O/cfg2_n$v.err || { echo "cfg2 n$v failed"; tail $O/cfg2_n$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/cfg2_n$v.json')); print('narrow=$v cfg2 loci/s', round(d['loci_per_s']), 'kernel ms', round(d['kernel_ms_per_step'],2), 'step ms', round(d['ms_per_step'],2))"
done
for v in 2 0; do
  WC_NARROW=$v timeout -k 10 300 python -u tools/cfg5_probe.py --loci 1024 --single 2 > $O/cfg5_n$v.log 2> $O/cfg5_n$v.err || { echo "cfg5 n$v failed"; tail $O/cfg5_n$v.err; exit 1; }
  echo "narrow=$v"; cat $O/cfg5_n$v.log
done
