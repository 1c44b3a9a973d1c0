#!/bin/bash
# GPU box: the vote-using suites on this tree, then cfg3 A/B old vs new
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_dual.py tests/test_gpu_builds.py tests/test_gpu_fullsize.py tests/test_priority_extras.py tests/test_gpu_single.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
bash tools/ab_libs.sh $1 cfg3 2 old new
