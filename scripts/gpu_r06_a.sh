# r6 a: the re-sort's multi-pass path (verdict r5 item 1). Re-sort and path-independence tests (C5 and the
# C5/8-rank shape over 300 steps: no whole-list range) and the Model R contact tests (cell skipping), C3 bench,
# C5 strong at 200 steps, a 200-step C5 kernel trace, the small-N timings.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06a; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_resort.py tests/test_gpu_path_independence.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_contact_team.py tests/test_gpu_shipped_bonds.py -m gpu -v -s -p no:cacheprovider --timeout=300 --timeout-method thread -x > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|shape|_resort" $O/pytest.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1; rc=$?; tail -8 $O/small_n.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_C3.log 2>&1; rc=$?
echo "bench C3 rc=$rc"; tail -c 1500 $O/bench_C3.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --strong --config C5 --no-cpu-baseline > $O/bench_C5.log 2>&1; rc=$?
echo "bench C5 rc=$rc"; tail -c 1500 $O/bench_C5.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/c5tr" -o run --output-format csv -- python3 scripts/run_steps.py --config C5 --steps 200 --warmup 0 > $O/c5tr.log 2>&1; rc=$?
f2=$(find $O/c5tr -name "*kernel_trace.csv" | head -1); python3 scripts/trace_kstats.py "$f2" 100000 2>&1 | head -12
exit $rc
