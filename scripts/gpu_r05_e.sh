# Round 5: the one-launch Model R step — its bit-identity and parity tests, then small-N timing and traces.
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05e; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v -s -m gpu --timeout 300 --timeout-method thread tests/test_gpu_fused.py \
  tests/test_gpu_parity.py tests/test_gpu_adhesion.py tests/test_gpu_resort.py tests/test_gpu_small.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E " passed| failed|FAILED|ERROR" $O/pytest.log | tail -15
[ $rc -ne 0 ] && { grep -B5 -A30 "Error\|FAILED\|assert" $O/pytest.log | tail -60; exit $rc; }
timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1; echo "small-N rc=$?"; grep -v amdgpu.ids $O/small_n.log
timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/r4096" -o run --output-format csv -- python3 scripts/run_steps.py --model-r 4096 --steps 300 > $O/r4096.log 2>&1; echo "R trace rc=$?"
f=$(find $O/r4096 -name "*kernel_trace.csv" | head -1); python3 scripts/trace_window.py "$f" 300 k_contact_fused
timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/c1" -o run --output-format csv -- python3 scripts/run_steps.py --config C1 --steps 300 > $O/c1.log 2>&1; echo "C1 trace rc=$?"
f=$(find $O/c1 -name "*kernel_trace.csv" | head -1); python3 scripts/trace_window.py "$f" 300 k_density_fused
exit 0
