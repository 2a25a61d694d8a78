# r6 c: re-sort tests and the C3 bench with direct cell shares; the comm stream's CU reservation (verdict r5 item 3). Which CUs a stream CU-mask bit enables
# (scripts/micro/cu_mask_probe), then the per-slab overhead with own comm streams (SPH_DEBUG_SERIAL_GROUP=2) at
# N = 2, 4 and an N = 4 kernel trace's comm slack, without and with the interior force pass on a CU-masked stream
# that leaves 8 CUs to the comm kernels (two candidate bit sets: one per XCD if the mask interleaves XCDs, or one per
# XCD if it is XCD-major).
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06c; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_resort.py tests/test_gpu_path_independence.py -m gpu -v -s -p no:cacheprovider --timeout=300 --timeout-method thread -x > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|'shape'|_resort" $O/pytest.log | tail -6
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --steps 200 --warmup 20 --no-cpu-baseline > $O/bench_C3.log 2>&1; rc=$?
echo "bench C3 rc=$rc"; python3 -c "
import json,sys
for l in open('$O/bench_C3.log'):
    if l.startswith('{') and 'metric' in l:
        d=json.loads(l); print(d['ms_per_step'], d.get('ms_per_step_mid_collapse'), d['kernels_ms_per_step'], d.get('kernels_ms_per_step_mid_collapse'))"
[ $rc -ne 0 ] && exit $rc
timeout -k 10 60 ./scripts/micro/cu_mask_probe > $O/cu_mask_probe.log 2>&1; rc=$?; cat $O/cu_mask_probe.log
[ $rc -ne 0 ] && exit $rc
i=0
for ex in "" "0,1,2,3,4,5,6,7" "0,32,64,96,128,160,192,224"; do
  i=$((i+1))
  if [ -n "$ex" ]; then export SPH_INTERIOR_CU_EXCLUDE="$ex"; else unset SPH_INTERIOR_CU_EXCLUDE; fi
  echo "== exclude [$ex]"
  GPU_MAX_HW_QUEUES=16 timeout -k 10 300 python -u scripts/slab_overhead.py 2,4 100 --no-concurrent --own-comm > $O/overhead_own_$i.log 2>&1; rc=$?
  grep world $O/overhead_own_$i.log; [ $rc -ne 0 ] && { tail -5 $O/overhead_own_$i.log; exit $rc; }
  export GPU_MAX_HW_QUEUES=16 SPH_DEBUG_SERIAL_GROUP=2
  timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/so4_$i" -o run --output-format csv -- python3 scripts/slab_trace.py 4 30 > $O/so4_$i.log 2>&1; rc=$?
  unset GPU_MAX_HW_QUEUES SPH_DEBUG_SERIAL_GROUP
  [ $rc -ne 0 ] && { tail -20 $O/so4_$i.log; exit $rc; }
  f=$(find $O/so4_$i -name "*kernel_trace.csv" | head -1)
  python3 scripts/comm_slack.py "$f" 4 20
done
exit 0
