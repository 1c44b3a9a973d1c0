set -o pipefail
O=gpurun_out/r02u
mkdir -p $O
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg3 --loci 768 --out $O/ph_cfg3 > $O/ph_cfg3.log 2>&1; echo "ph cfg3 rc=$?"
