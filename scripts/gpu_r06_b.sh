# r6 b: k_mv_rank with 32,768-slot ranges and 65,536-cell shares (staged keys, passes of 8,192 cells): re-sort and
# path-independence tests, the Model R tests (compacted contact bodies), small-N timings, C3 bench, C5 strong at 200
# and 1,000 steps, a 200-step C5 kernel trace.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06b; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests/test_gpu_resort.py tests/test_gpu_path_independence.py tests/test_gpu_parity.py tests/test_gpu_fused.py tests/test_gpu_small.py tests/test_gpu_contact_team.py tests/test_gpu_shipped_bonds.py tests/test_gpu_parity_headline.py tests/test_gpu_slab.py -m gpu -v -s -p no:cacheprovider --timeout=300 --timeout-method thread -x > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|'shape'|_resort" $O/pytest.log | tail -12
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1; rc=$?; tail -5 $O/small_n.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_C3.log 2>&1; rc=$?
echo "bench C3 rc=$rc"; python3 -c "
import json,sys
for l in open('$O/bench_C3.log'):
    if l.startswith('{') and 'metric' in l:
        d=json.loads(l); print(d['ms_per_step'], d.get('ms_per_step_mid_collapse'), d['kernels_ms_per_step'], d.get('kernels_ms_per_step_mid_collapse'), d['resort_counts'])"
[ $rc -ne 0 ] && exit $rc
for st in 200 1000; do
timeout -k 10 400 python -u bench.py --strong --config C5 --no-cpu-baseline --steps $st > $O/bench_C5_$st.log 2>&1; rc=$?
echo "bench C5 $st rc=$rc"; python3 -c "
import json,sys
for l in open('$O/bench_C5_$st.log'):
    if l.startswith('{') and 'metric' in l:
        d=json.loads(l); print(d['steps'], d['ms_per_step'], d['kernels_ms_per_step'], d['resort_counts'], d.get('kernels_sum_over_gpu_event'))"
[ $rc -ne 0 ] && exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/c5tr" -o run --output-format csv -- python3 scripts/run_steps.py --config C5 --steps 200 --warmup 0 > $O/c5tr.log 2>&1; rc=$?
f2=$(find $O/c5tr -name "*kernel_trace.csv" | head -1); python3 scripts/trace_kstats.py "$f2" 100000 2>&1 | head -6
exit $rc
