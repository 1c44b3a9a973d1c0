set -o pipefail
export TMPDIR=/tmp
bash tools/profile_round.sh r02g --workload cfg3 --loci 768 > gpurun_out/prof_r02g.log 2>&1 || { echo "profile failed"; tail gpurun_out/prof_r02g.log; exit 1; }
echo done
