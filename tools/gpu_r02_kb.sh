set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_kb
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu --no-e2e > $O/cfg2.json 2> $O/cfg2.err || { echo "cfg2 failed"; tail $O/cfg2.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg2.json')); print('cfg2 loci/s', round(d['loci_per_s']), 'kernel ms', round(d['kernel_ms_per_step'],2), 'step ms', round(d['ms_per_step'],2))"
WC_HOST_TIMING=1 timeout -k 10 200 python -u tools/host_profile.py > $O/host_timing.txt 2>&1 || { echo "host timing failed"; exit 1; }
grep wall_ms $O/host_timing.txt
