# Round 6 final measurement (second bundle, after the small-N latency work), part 2: PMC passes and GRBM clocks for the final code objects (stamped with the
# device-code hash), then the driver's default bench line, which reads them for its roofline.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/fin7; mkdir -p $O
( while true; do date >> $O/heartbeat2; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
export TMPDIR=/tmp
bash scripts/gpu_pmc.sh > $O/pmc.log 2>&1; rc=$?
echo "pmc rc=$rc"; tail -3 $O/pmc.log
[ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_C3.json C3 > gpurun_out/pmc_summary.log 2>&1
echo "pmc_summary rc=$?"
bash scripts/gpu_clock.sh > gpurun_out/clock.log 2>&1; echo "clock rc=$?"; tail -3 gpurun_out/clock.log
cp gpurun_out/pmc_C3.json profiles/pmc_C3.json; cp gpurun_out/clock/clock.json profiles/clock_r06.json 2>/dev/null
timeout -k 10 400 python bench.py > $O/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 $O/bench.log | cut -c 1-600
exit $rc
