# C1 small-N step: the Model S small-path tests, then C1 timing and a C1 kernel trace.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05i; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_small.py tests/test_gpu_parity.py tests/test_gpu_path_independence.py tests/test_gpu_resort.py -m gpu -q -p no:cacheprovider --timeout=300 --timeout-method thread -x > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -8
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1; rc=$?; grep "S C1" $O/small_n.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/c1tr" -o run --output-format csv -- python3 scripts/run_steps.py --config C1 --steps 300 --warmup 20 > $O/c1tr.log 2>&1; rc=$?
f2=$(find $O/c1tr -name "*kernel_trace.csv" | head -1); python3 scripts/trace_window.py "$f2" 200 k_density_fused 2>&1 | tail -4
exit $rc
