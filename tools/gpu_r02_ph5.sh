set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_ph5
mkdir -p $O
WC_HOST_TIMING=1 timeout -k 10 200 python -u tools/host_profile.py > $O/host_timing.txt 2>&1 || { echo "host timing failed"; tail $O/host_timing.txt; exit 1; }
grep "\[wc\]" $O/host_timing.txt | tail -3; grep wall_ms $O/host_timing.txt
WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 400 python -u tools/phase_run.py --workload cfg5-hpc --loci 1024 --out $O/ph > $O/phase.log 2>&1 || { echo "phase failed"; tail $O/phase.log; exit 1; }
cat $O/phase.log | tail -60
