set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_ph2
mkdir -p $O
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 300 python -u tools/phase_run.py --workload cfg2 --loci 1000 --out $O/ph > $O/phase.log 2>&1 || { echo "phase failed"; tail $O/phase.log; exit 1; }
python -c "import json; d=json.load(open('$O/ph/report.json')); [print(k, d[k]) for k in ('kernel_ms','chains','sub_cycles_per_chain','block_cycles_per_chain','phase_share','heaviest_alone_kernel_ms')]"
