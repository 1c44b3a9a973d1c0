set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_host
mkdir -p $O
WC_HOST_TIMING=1 timeout -k 10 200 python -u tools/host_profile.py > $O/host_timing.txt 2>&1 || { echo "host timing failed"; exit 1; }
grep "\[wc\]" $O/host_timing.txt | tail -2; grep wall_ms $O/host_timing.txt; grep -A16 "Ordered by" $O/host_timing.txt | head -18
