#!/bin/bash
# GPU box: dual/priority suites, one-sub-problem timing, then the cfg5 PMC
# passes (kernel trace, FETCH_SIZE, WRITE_SIZE, issue view) of the wave kernel
export TMPDIR=/tmp
T=$1
O=gpurun_out/$T
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dual.py tests/test_priority_extras.py tests/test_gpu_builds.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for seed in 5949 1525; do
  timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed $seed > $O/s$seed.log 2>&1 || exit 1
  echo $seed $(grep -o '"us_per_pop": [0-9.]*' $O/s$seed.log)
done
PASSES="kt fetch write sq1" bash tools/profile_round.sh ${T} --workload cfg5 --loci 10000 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -2 $O/prof.log
