set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02x
mkdir -p $O
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SMEM --output-format csv -d $O/p1 -o run -- python3 tools/one_locus.py > $O/p1.log 2>&1; echo "p1 rc=$?"
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_BRANCH SQ_INSTS_VMEM_WR SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS --output-format csv -d $O/p2 -o run -- python3 tools/one_locus.py > $O/p2.log 2>&1; echo "p2 rc=$?"
tail -1 $O/p1.log
python3 - <<'PY'
import csv, collections
for p in ("p1", "p2"):
    rows = [r for r in csv.DictReader(open(f"gpurun_out/r02x/{p}/run_counter_collection.csv")) if "dual_engine" in r["Kernel_Name"]]
    last = max(int(r["Dispatch_Id"]) for r in rows)
    s = collections.defaultdict(float)
    for r in rows:
        if int(r["Dispatch_Id"]) == last:
            s[r["Counter_Name"]] += float(r["Counter_Value"])
    print(p, dict(s))
PY
