# 2-wave low-latency build for small launches: parity suite, latency workloads
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_ll
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_builds.py -x -q --timeout 120 --timeout-method thread > $O/pytest_builds.log 2>&1 || { echo "build tests failed"; tail -30 $O/pytest_builds.log; exit 1; }
tail -1 $O/pytest_builds.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
for v in 1 0; do
  WC_LOWLAT=$v timeout -k 10 300 python -u bench.py --workload cfg2-latency --steps 10 --warmup 2 --no-cpu > $O/lat_$v.json 2> $O/lat_$v.err || { echo "lat $v failed"; tail $O/lat_$v.err; exit 1; }
  python -c "import json; d=json.load(open('$O/lat_$v.json')); print('lowlat=$v cfg2-latency ms', round(d['ms_per_step'],2), 'kernel', round(d['kernel_ms_per_step'],2))"
done
timeout -k 10 300 python -u bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 failed"; tail $O/cfg4.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg4.json')); print('cfg4 s', round(d['ms_per_step']/1e3,2))"
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > $O/cfg2.json 2> $O/cfg2.err || { echo "cfg2 failed"; tail $O/cfg2.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg2.json')); print('cfg2 loci/s', round(d['loci_per_s']), 'kernel ms', round(d['kernel_ms_per_step'],2))"
