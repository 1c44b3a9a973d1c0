set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02z
mkdir -p $O
export WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_w2.so
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e > $O/write_bench.json 2> $O/write.err; echo "w rc=$?"
timeout -s KILL 240 rocprofv3 --pmc SQ_INSTS_VMEM_WR SQ_WAVES --output-format csv -d $O/sq -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu --no-e2e > $O/sq_bench.json 2> $O/sq.err; echo "sq rc=$?"
python3 - <<'PY'
import csv, collections
for p in ("write", "sq"):
    s = collections.defaultdict(float)
    for r in csv.DictReader(open(f"gpurun_out/r02z/{p}/run_counter_collection.csv")):
        if "engine_kernel" in r["Kernel_Name"]:
            s[r["Counter_Name"]] += float(r["Counter_Value"])
    print(p, dict(s))
PY
python3 -c "import json; d=json.load(open('gpurun_out/r02z/write_bench.json')); print('w2 kernel ms', d['kernel_ms_per_step'], d['loci_per_s'])"
