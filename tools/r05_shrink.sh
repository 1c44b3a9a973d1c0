#!/bin/bash
# GPU box: priority suites, then cfg4's sub-problem path and bench line
export TMPDIR=/tmp
O=gpurun_out/$1
mkdir -p $O
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_priority_extras.py tests/test_gpu_fullsize.py tests/test_gpu_dual.py tests/test_gpu_service.py -m gpu > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
WC_LAUNCH_LOG=1 timeout -k 10 300 python3 -u tools/cfg4_path.py --out $O > $O/c4p.log 2>&1 || { tail -20 $O/c4p.log; exit 1; }
grep -v amdgpu $O/c4p.log | grep -v "\[wc\] launch\|\[wc\] done" | head -3
grep "stream launch" $O/c4p.log | head -5
