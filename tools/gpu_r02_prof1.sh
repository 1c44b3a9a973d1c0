# cfg2: host-side split of a bench step, then the profile passes of the current kernel.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r02_prof1
mkdir -p $O
timeout -k 10 200 python -u tools/host_profile.py > $O/host_profile.txt 2>&1 || { echo "host_profile failed"; tail $O/host_profile.txt; exit 1; }
head -40 $O/host_profile.txt
bash tools/profile_round.sh r02c || exit 1
echo prof done
