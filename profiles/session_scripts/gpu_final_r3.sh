#!/bin/bash
# Round 3 final profiles on the committed build: rocprofv3 kernel traces + calibrated HBM traffic
# (separate FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md §HBM) of every bench
# configuration -- c3, c2, c4, c5 (round 6) and the strong-scaling shards 2048 / 1024 / 512 -- into
# profiles/pmc_traffic.json stamped with the KKT source hash (bench.py drops a stale entry).
# OUT=... CONFIGS="c3 c2 ..." to run a subset.
R="${GRAFT_REPO_ROOT:-/root/repo}"
cd "$R"; O=gpurun_out/${OUT:-final_r3}; mkdir -p $O
export TMPDIR=/tmp
run() { local t=$1; local log=$2; shift 2; timeout -k 10 "$t" "$@" > "$O/$log" 2>&1; local rc=$?; echo "rc=$rc $log"; tail -1 "$O/$log" | cut -c1-300; if [ $rc -ne 0 ]; then exit $rc; fi; }
cp profiles/pmc_traffic.json $O/pmc_traffic.json
for c in ${CONFIGS:-c3 c2 c4 c5 s2048 s1024 s512}; do
  case $c in
    c3) A="--steps 20 --warmup 2"; KEY=cartpole_N200_B4096; K=kkt_scan ;;
    c2) A="--problem pendulum --horizon 100 --batch 1024 --steps 50 --warmup 5"; KEY=pendulum_N100_B1024; K=kkt_scan ;;
    c4) A="--problem linear8 --horizon 512 --batch 16384 --lanes 1 --steps 5 --warmup 1"; KEY=linear8_N512_B16384; K=kkt_group8 ;;
    c5) A="--batch 8192 --steps 20 --warmup 2"; KEY=cartpole_N200_B8192; K=kkt_scan ;;
    s2048) A="--batch 2048 --steps 50 --warmup 5"; KEY=cartpole_N200_B2048; K=kkt_scan ;;
    s1024) A="--batch 1024 --steps 50 --warmup 5"; KEY=cartpole_N200_B1024; K=kkt_scan ;;
    s512) A="--batch 512 --steps 50 --warmup 5"; KEY=cartpole_N200_B512; K=kkt_scan ;;
  esac
  A="$A --no-cpu --no-ipm"
  run 240 ${c}_trace.log rocprofv3 --kernel-trace --stats --output-format csv -d "$R/$O/${c}_trace" -o run -- python "$R/bench.py" $A
  run 120 ${c}_fetch.log timeout -s KILL 110 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$R/$O/${c}_fetch" -o run -- python "$R/bench.py" $A
  run 120 ${c}_write.log timeout -s KILL 110 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$R/$O/${c}_write" -o run -- python "$R/bench.py" $A
  python tools/pmc_traffic.py $O/${c}_fetch/run_counter_collection.csv $O/${c}_write/run_counter_collection.csv $KEY $O/pmc_traffic.json $K > $O/${c}_traffic.log 2>&1 || exit 1
  tail -1 $O/${c}_traffic.log
done
