# Round measurement (after the GPU tests): rocprofv3 kernel stats of the bench command, PMC passes (one counter group
# per run) and GRBM clock passes summarised into files stamped with the library's device-code hash (bench.py uses them
# only for the same code objects), the default bench line, and the slab step's per-slab cost.
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/slabtrace; export TMPDIR=/tmp
R=${ROUND:-r04}
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prof" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --mid-steps 0 --no-cpu-baseline > gpurun_out/prof.log 2>&1; rc=$?
echo "rocprof rc=$rc"; tail -1 gpurun_out/prof.log | cut -c 1-200
[ $rc -ne 0 ] && exit $rc
bash scripts/gpu_pmc.sh; rc=$?
echo "pmc rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 scripts/pmc_summary.py gpurun_out/pmc gpurun_out/pmc_C3.json C3 > gpurun_out/pmc_summary.log 2>&1
echo "pmc_summary rc=$?"
bash scripts/gpu_clock.sh > gpurun_out/clock.log 2>&1; echo "clock rc=$?"; tail -3 gpurun_out/clock.log
cp gpurun_out/pmc_C3.json profiles/pmc_C3.json; cp gpurun_out/clock/clock.json profiles/clock_$R.json 2>/dev/null
timeout -k 10 400 python bench.py > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -1 gpurun_out/bench.log | cut -c 1-300
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u scripts/slab_overhead.py 2,4,8 100 --no-concurrent > gpurun_out/slab_overhead.log 2>&1; echo "slab_overhead rc=$?"; tail -3 gpurun_out/slab_overhead.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/slabtrace/k4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/slab_trace.py" 4 30 > gpurun_out/slabtrace/k4.log 2>&1; echo "trace rc=$?"
exit 0
