# Round measurement: GPU tests, smoke, default bench line, rocprofv3 kernel stats of the same bench
# command, PMC passes (one counter group per run) and GRBM clock passes, both summarised into files
# stamped with the library's device-code hash (bench.py uses them only for the same code objects).
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout=600 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED" gpurun_out/pytest_gpu.log | tail -6
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
# the profiled command: the driver's bench (steps 20, warmup 5) without the mid-collapse advance, whose
# 5,000 untimed steps would otherwise dominate every kernel's average
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --mid-steps 0 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log | cut -c 1-300
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_pmc.sh; rc=$?
echo "pmc rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_C3.json C3 > gpurun_out/pmc_summary.log 2>&1
echo "pmc_summary rc=$?"
bash scripts/gpu_clock.sh > gpurun_out/clock.log 2>&1; echo "clock rc=$?"; tail -3 gpurun_out/clock.log
# the driver's default bench line, after the counter files exist (its roofline reads them)
cp gpurun_out/pmc_C3.json profiles/pmc_C3.json; cp gpurun_out/clock/clock.json profiles/clock_${ROUND:-r04}.json 2>/dev/null
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c 1-600
exit 0
