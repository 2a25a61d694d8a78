# Round 5: re-sort check — the re-sort bit-identity tests, the bench line (rest + mid-collapse), a mid-collapse trace.
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05c; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
python -c "import torch; print(torch.__version__, flush=True)"
timeout -k 10 600 python -u -m pytest -x -v -s -m gpu --timeout 300 --timeout-method thread tests/ > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E " passed| failed|FAILED|ERROR" $O/pytest.log | tail -15
[ $rc -ne 0 ] && { grep -B5 -A40 "Error\|FAILED\|assert" $O/pytest.log | tail -80; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc"; tail -c 700 $O/bench.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/mid" -o run --output-format csv -- python3 scripts/mid_trace.py > $O/mid.log 2>&1; rc=$?
echo "mid trace rc=$rc"; grep -v amdgpu.ids $O/mid.log; [ $rc -ne 0 ] && exit $rc
f=$(find $O/mid -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_window.py "$f" 200 k_density_tiled
timeout -k 10 300 python scripts/rank_probe.py --steps 4 > $O/probe.log 2>&1; echo "probe rc=$?"; grep -v amdgpu.ids $O/probe.log | cut -c1-400
exit 0
