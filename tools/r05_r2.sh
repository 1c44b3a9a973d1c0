#!/bin/bash
# GPU box: dual suites (votes / capacity-check changes), then the full-read
# level alone: 5949 (56 reads, R=1) and 1525 (80 reads, R=2), wave vs block,
# and phase profiles of the wave engine on both
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dual.py tests/test_priority_extras.py tests/test_gpu_builds.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for seed in 5949 1525; do
  for eng in 1 0; do
    WC_WAVE=$eng timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed $seed > $O/s${seed}_$eng.log 2>&1 || exit 1
    echo $seed $eng $(grep us_per_pop $O/s${seed}_$eng.log)
  done
  WC_WAVE=1 WAFFLE_CON_LIB=$PWD/waffle_con_amd/libwaffle_con_prof.so timeout -k 10 200 python3 -u tools/one_sub.py --workload cfg5-full --seed $seed --phases /tmp/ph_$seed.txt > $O/ph_$seed.log 2>&1 || exit 1
  grep -v amdgpu $O/ph_$seed.log | tail -1
done
