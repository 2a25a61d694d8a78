# Round 6 final measurement (second bundle, after the small-N latency work), part 1: the whole GPU suite, smoke, the rocprofv3 kernel stats of the driver's bench command.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/fin7; mkdir -p $O
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 --timeout-method thread -rA -s > $O/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" $O/pytest_gpu.log | tail -6
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 $O/smoke.log
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --mid-steps 0 --no-cpu-baseline > $O/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -1 $O/prof.log | cut -c 1-300
exit $rc
