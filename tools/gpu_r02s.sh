set -o pipefail
O=gpurun_out/r02s
mkdir -p $O
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg5-hpc --loci 1024 --out $O/ph_cfg5 > $O/ph_cfg5.log 2>&1; echo "ph cfg5 rc=$?"
