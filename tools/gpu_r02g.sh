set -o pipefail
mkdir -p gpurun_out/r02g
timeout -k 10 600 python -u -m pytest tests -m gpu -v --maxfail=5 --timeout 170 --timeout-method thread -k "not cfg4_full" > gpurun_out/r02g/gpu_tests.log 2>&1
echo "tests rc=$?"
tail -3 gpurun_out/r02g/gpu_tests.log
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg3 --loci 256 --out gpurun_out/r02g/ph_cfg3 > gpurun_out/r02g/ph_cfg3.log 2>&1; echo "ph cfg3 rc=$?"
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python -u tools/phase_run.py --workload cfg5-hpc --loci 1024 --out gpurun_out/r02g/ph_cfg5 > gpurun_out/r02g/ph_cfg5.log 2>&1; echo "ph cfg5 rc=$?"
bash tools/profile_round.sh r02
