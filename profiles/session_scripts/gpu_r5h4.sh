#!/bin/bash
# Solver state after the first K solves of the c3 persistent solve vs its remaining solves
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-r5h4}; mkdir -p $O
export TMPDIR=/tmp
PROBE_KS=${PROBE_KS:-1,2,3,5,10} timeout -k 10 180 python tools/predict_probe.py $O > $O/predict.log 2>&1; rc=$?; tail -4 $O/predict.log; exit $rc
