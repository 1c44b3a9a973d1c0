#!/bin/bash
# GPU box: the dual diagnostic on the lane-parallel vote-count variants, then cfg3 A/B
export TMPDIR=/tmp
bash tools/r05_vd.sh $1 lp1 lp2 && bash tools/ab_libs.sh $1 cfg3 2 lp0 lp1 lp2
