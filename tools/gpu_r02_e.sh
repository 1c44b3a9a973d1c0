set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_e
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
WC_HOST_TIMING=1 timeout -k 10 200 python -u tools/host_profile.py > $O/host_timing.txt 2>&1 || { echo "host timing failed"; exit 1; }
grep "\[wc\]" $O/host_timing.txt | tail -2; grep wall_ms $O/host_timing.txt; grep -A12 "Ordered by" $O/host_timing.txt | head -14
timeout -k 10 400 python -u bench.py > $O/cfg2.json 2> $O/cfg2.err || { echo "cfg2 failed"; tail $O/cfg2.err; exit 1; }
python -c "import json; d=json.load(open('$O/cfg2.json')); print('cfg2 loci/s', round(d['loci_per_s']), 'kernel ms', round(d['kernel_ms_per_step'],2), 'step ms', round(d['ms_per_step'],2), 'median', round(d['ms_per_step_median'],2), 'cpu x', round(d['gpu_vs_cpu_loci'],1), 'e2e', round(d['e2e_loci_per_s']))"
bash tools/profile_round.sh r02e > $O/prof.log 2>&1 || { echo "profile failed"; tail $O/prof.log; exit 1; }
echo profile done
