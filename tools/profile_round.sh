#!/bin/bash
# Profiles the bench workload on the GPU box (run through gpurun):
#   1. kernel trace + stats (per-kernel durations)
#   2. PMC pass FETCH_SIZE, 3. PMC pass WRITE_SIZE (separate passes: TCC slots)
# Outputs under gpurun_out/prof_<tag>/; tools/pmc_summary.py condenses them.
set -e
TAG=${1:-r01}
LOCI=${LOCI:-1000}
export TMPDIR=/tmp
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 bench.py --loci $LOCI --steps 3 --warmup 1 --no-cpu > $OUT/kt_bench.json
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- \
  python3 bench.py --loci $LOCI --steps 1 --warmup 0 --no-cpu > $OUT/fetch_bench.json
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- \
  python3 bench.py --loci $LOCI --steps 1 --warmup 0 --no-cpu > $OUT/write_bench.json
echo "profile $TAG done"
