set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_c4b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 failed"; tail $O/cfg4.err; exit 1; }
grep "stream launch\|done" $O/cfg4.err | head -10
python -c "import json; d=json.load(open('$O/cfg4.json')); print('cfg4 s', round(d['ms_per_step']/1e3,2), 'kernel s', round(d['kernel_ms_per_step']/1e3,2))"
timeout -k 10 300 python -u bench.py --workload cfg5 --loci 4096 --steps 1 --warmup 0 --no-cpu > $O/cfg5_4096.json 2> $O/cfg5_4096.err || { echo "cfg5 4096 failed"; tail $O/cfg5_4096.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg5_4096.json')); print('cfg5 4096 loci/s', round(d['loci_per_s'],1))"
