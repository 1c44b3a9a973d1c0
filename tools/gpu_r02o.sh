set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02o
mkdir -p $O
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $O/ic -o run -- python3 bench.py --workload cfg3 --loci 768 --steps 1 --warmup 0 --no-cpu --no-e2e > $O/ic_bench.json 2> $O/ic_bench.err; echo "ic rc=$?"
python3 - <<'PY'
import csv, collections
s = collections.defaultdict(float)
for r in csv.DictReader(open("gpurun_out/r02o/ic/run_counter_collection.csv")):
    if "dual_engine" in r["Kernel_Name"]:
        s[r["Counter_Name"]] += float(r["Counter_Value"])
print(dict(s))
PY
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_Os.so timeout -k 10 200 python -u bench.py --workload cfg3 --loci 768 --steps 1 --warmup 1 --no-cpu --no-e2e > $O/cfg3_Os.json 2> $O/cfg3_Os.err; echo "Os rc=$?"
python -c "import json; d=json.load(open('$O/cfg3_Os.json')); print('Os cfg3 loci/s', d['loci_per_s'], 'kernel ms', d['kernel_ms_per_step'])"
