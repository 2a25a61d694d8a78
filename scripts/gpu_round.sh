# Round measurement: GPU tests, smoke, default bench line, rocprofv3 kernel stats of the same
# bench command, and PMC passes (one counter group per run) summarised for bench's roofline.traffic.
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -m gpu -q -p no:cacheprovider --timeout=300 > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; tail -2 gpurun_out/pytest_gpu.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?
echo "smoke rc=$rc"; tail -2 gpurun_out/smoke.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
export TMPDIR=/tmp
# the profiled command: the driver's bench (steps 20, warmup 5) without the mid-collapse advance, whose
# 5,000 untimed steps would otherwise dominate every kernel's average (the line's roofline.kernel_avg_us
# is over the timed region only)
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --mid-steps 0 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_pmc.sh; rc=$?
echo "pmc rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_C3.json C3 > gpurun_out/pmc_summary.log 2>&1
echo "pmc_summary rc=$?"
exit 0
