# overlapped harvest + bulk decode, narrow dual default, bounded stream publication
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_n2
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -u bench.py --steps 5 --warmup 1 --no-cpu > $O/cfg2.json 2> $O/cfg2.err || { echo "cfg2 failed"; tail $O/cfg2.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg2.json')); print('cfg2 loci/s', round(d['loci_per_s']), 'kernel ms', round(d['kernel_ms_per_step'],2), 'step ms', round(d['ms_per_step'],2), 'e2e', round(d['e2e_loci_per_s']))"
WC_HOST_TIMING=1 timeout -k 10 200 python -u tools/host_profile.py > $O/host_timing.txt 2>&1 || { echo "host timing failed"; exit 1; }
grep "\[wc\]" $O/host_timing.txt | tail -2; grep wall_ms $O/host_timing.txt
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u tools/cfg5_probe.py --loci 1024 --single 0 > $O/cfg5.log 2> $O/cfg5.err || { echo "cfg5 failed"; tail $O/cfg5.err; exit 1; }
cat $O/cfg5.log; grep "stream:" $O/cfg5.err | tail -4
WC_LAUNCH_LOG=1 timeout -k 10 400 python -u bench.py --workload cfg5 --loci 4096 --steps 1 --warmup 0 --no-cpu > $O/cfg5_4096.json 2> $O/cfg5_4096.err || { echo "cfg5 4096 failed"; tail $O/cfg5_4096.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg5_4096.json')); print('cfg5 4096 loci/s', round(d['loci_per_s'],1), 'step s', round(d['ms_per_step']/1e3,2))"; grep "stream:" $O/cfg5_4096.err | tail -6
