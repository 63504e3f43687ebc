#!/bin/bash
# Round 5: issue-priority experiment (ablation bits 7 / 8: s_setprio of the memory phases vs the
# scan phase), graph-replayed, same build for every variant.  The bits were removed after this
# run (profiles/r05/setprio_rejected/); rerunning needs them back in kkt_scan_impl.h.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/r5s; mkdir -p $O
export TMPDIR=/tmp
export ABLATE_VARIANTS='{"full": 0, "prio_mem": 128, "prio_scan": 256, "prio_p1p2": 384}'
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-600; if [ $rc -ne 0 ]; then exit $rc; fi; }
run 240 c3.log python tools/kkt_ablate.py cartpole 200 4096 32
run 200 s1024.log python tools/kkt_ablate.py cartpole 200 1024 64
run 200 s512.log python tools/kkt_ablate.py cartpole 200 512 128
run 200 c2.log python tools/kkt_ablate.py pendulum 100 1024 64
run 240 c3b.log python tools/kkt_ablate.py cartpole 200 4096 32
