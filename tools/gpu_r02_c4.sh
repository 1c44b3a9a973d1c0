set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_c4
mkdir -p $O
WC_LAUNCH_LOG=1 timeout -k 10 300 python -u bench.py --workload cfg4 --steps 1 --warmup 0 --no-cpu > $O/cfg4.json 2> $O/cfg4.err || { echo "cfg4 failed"; tail $O/cfg4.err; exit 1; }
grep "\[wc\]" $O/cfg4.err | head -30
python -c "import json; d=json.load(open('$O/cfg4.json')); print('cfg4 s', round(d['ms_per_step']/1e3,2), 'kernel s', round(d['kernel_ms_per_step']/1e3,2))"
