set -o pipefail
O=gpurun_out/r02y
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -v --timeout 170 --timeout-method thread -k "not cfg4_full" > $O/tests.log 2>&1
echo "tests rc=$?"
tail -2 $O/tests.log
timeout -k 10 300 python -u bench.py --steps 2 --warmup 1 --no-cpu --no-e2e > $O/cfg2.json 2> $O/cfg2.err || { echo "cfg2 failed"; exit 1; }
python -c "import json; d=json.load(open('$O/cfg2.json')); print('cfg2 loci/s', d['loci_per_s'], 'kernel ms', d['kernel_ms_per_step'])"
timeout -k 10 200 python -u bench.py --workload cfg3 --loci 768 --steps 1 --warmup 1 --no-cpu --no-e2e > $O/cfg3.json 2> $O/cfg3.err || { echo "cfg3 failed"; exit 1; }
python -c "import json; d=json.load(open('$O/cfg3.json')); print('cfg3 loci/s', d['loci_per_s'], 'kernel ms', d['kernel_ms_per_step'])"
timeout -k 10 300 python -u tools/priority_bench.py --loci 1024 --cpu-loci 4 > $O/prio.json 2> $O/prio.err || { echo "prio failed"; exit 1; }
cat $O/prio.json
