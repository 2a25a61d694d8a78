# Round 5, first box: the RCCL failure paths and the moved flags' all-reduce (tests), the 2/4/8-rank RCCL rehearsal,
# the serialised per-slab overhead, kernel traces of the slab step at N = 4 / 8 and of C3 mid-collapse.
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05a; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
python -c "import torch; print(torch.__version__, flush=True)"
part1() {
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread tests/test_gpu_rccl.py > $O/pytest_rccl.log 2>&1
echo "rccl tests rc=$?"; grep -E "PASSED|FAILED|ERROR|rank . stderr|step [0-9]+ issued" $O/pytest_rccl.log | tail -12
timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1; echo "small-N rc=$?"; cat $O/small_n.log
timeout -k 10 600 python -u -m pytest -x -v -s --timeout 300 --timeout-method thread \
  tests/test_gpu_bench_launch.py tests/test_gpu_multi.py > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|PASSED|FAILED|ERROR" $O/pytest.log | tail -30
[ $rc -ne 0 ] && { tail -60 $O/pytest.log; exit $rc; }
RANKS="2 4 8" STEPS=60 WARMUP=10 LIMIT=300 bash scripts/gpu_rccl_rehearsal.sh > $O/rehearsal.log 2>&1; rc=$?
cat $O/rehearsal.log; [ $rc -ne 0 ] && exit $rc
exit 0
}
part2() {
timeout -k 10 300 python -u scripts/slab_overhead.py 2,4,8 100 --no-concurrent > $O/overhead.log 2>&1; rc=$?
cat $O/overhead.log; [ $rc -ne 0 ] && exit $rc
GPU_MAX_HW_QUEUES=12 timeout -k 10 300 python -u scripts/slab_overhead.py 2,4,8 100 --no-concurrent --own-comm > $O/overhead_own.log 2>&1; rc=$?
cat $O/overhead_own.log; [ $rc -ne 0 ] && exit $rc
for n in 4 8; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/st$n" -o run --output-format csv -- python3 scripts/slab_trace.py $n 30 > $O/st$n.log 2>&1; rc=$?
  echo "slab trace n=$n rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/st$n.log; exit $rc; }
  f=$(find $O/st$n -name "*kernel_trace.csv" | head -1)
  python3 scripts/trace_window.py "$f" $((30 * n)) k_density_tiled; python3 scripts/comm_slack.py "$f" $n 20
done
export GPU_MAX_HW_QUEUES=12 SPH_DEBUG_SERIAL_GROUP=2
timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/so8" -o run --output-format csv -- python3 scripts/slab_trace.py 8 30 > $O/so8.log 2>&1; rc=$?
echo "slab trace own comm n=8 rc=$rc"; [ $rc -ne 0 ] && { tail -20 $O/so8.log; exit $rc; }
f=$(find $O/so8 -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_window.py "$f" 240 k_density_tiled; python3 scripts/comm_slack.py "$f" 8 20
unset GPU_MAX_HW_QUEUES SPH_DEBUG_SERIAL_GROUP
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/$O/mid" -o run --output-format csv -- python3 scripts/mid_trace.py > $O/mid.log 2>&1; rc=$?
echo "mid trace rc=$rc"; cat $O/mid.log | grep -v amdgpu.ids; [ $rc -ne 0 ] && exit $rc
f=$(find $O/mid -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_window.py "$f" 200 k_density_tiled
exit 0
}
part${1:-1}
