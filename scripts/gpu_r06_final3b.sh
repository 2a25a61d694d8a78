# Round 6 final measurement (second bundle, after the small-N latency work), part 3: PMC passes of the strong configurations (C4, C5; profiles/pmc_C4.json,
# pmc_C5.json for their lines' traffic), C5 at 200 and 1,000 steps, the per-slab overhead (slabs serialised on one GPU,
# N = 2, 4, 8; own comm streams at N = 2, 4), and the rate table.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/fin7; mkdir -p $O
( while true; do date >> $O/heartbeat3; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
CONFIGS="C4 C5" bash scripts/gpu_pmc_strong.sh > $O/pmc_strong.log 2>&1; rc=$?
echo "pmc strong rc=$rc"; grep -E "rc=" $O/pmc_strong.log | tail -12
[ $rc -ne 0 ] && exit $rc
for st in 200 1000; do
  timeout -k 10 400 python -u bench.py --strong --config C5 --no-cpu-baseline --steps $st > $O/bench_C5_$st.log 2>&1; rc=$?
  echo "bench C5 $st rc=$rc"; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 python -u scripts/slab_overhead.py 2,4,8 100 --no-concurrent > $O/overhead.log 2>&1; rc=$?
grep world $O/overhead.log; [ $rc -ne 0 ] && exit $rc
GPU_MAX_HW_QUEUES=12 timeout -k 10 300 python -u scripts/slab_overhead.py 2,4 100 --no-concurrent --own-comm > $O/overhead_own.log 2>&1; rc=$?
grep world $O/overhead_own.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 600 python -u bench.py --table > $O/rate_table.log 2>&1; rc=$?
echo "table rc=$rc"; tail -3 $O/rate_table.log | cut -c 1-400
exit $rc
