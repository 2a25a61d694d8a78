# Round 5: the whole GPU suite, the bench line (rest + mid-collapse), a kernel trace mid-collapse with mover counts.
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05b; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
python -c "import torch; print(torch.__version__, flush=True)"
timeout -k 10 1000 python -u -m pytest -x -v -s -m gpu --timeout 300 --timeout-method thread tests/ > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E " passed| failed|FAILED|ERROR" $O/pytest.log | tail -15
[ $rc -ne 0 ] && { grep -B5 -A40 "Error\|FAILED\|assert" $O/pytest.log | tail -80; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline > $O/bench.log 2>&1; echo "bench rc=$?"; tail -c 1500 $O/bench.log
for sc in 0 1; do
  SPH_SCHED=$sc timeout -k 10 300 python bench.py --strong --config C5 --steps 20 --warmup 3 --no-cpu-baseline --mid-steps 0 > $O/bench_c5_sched$sc.log 2>&1; echo "C5 sched=$sc rc=$?"
  python3 -c "import json,sys; d=json.loads(open('$O/bench_c5_sched$sc.log').read().strip().splitlines()[-1]); print('C5 sched', $sc, d['ms_per_step'], d.get('kernels_ms_per_step'))"
done
timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/mid" -o run --output-format csv -- python3 scripts/mid_trace.py > $O/mid.log 2>&1; rc=$?
echo "mid trace rc=$rc"; grep -v amdgpu.ids $O/mid.log; [ $rc -ne 0 ] && exit $rc
f=$(find $O/mid -name "*kernel_trace.csv" | head -1)
python3 scripts/trace_window.py "$f" 200 k_density_tiled
timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1; echo "small-N rc=$?"; grep -v amdgpu.ids $O/small_n.log
timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/r4096" -o run --output-format csv -- python3 scripts/run_steps.py --model-r 4096 --steps 300 > $O/r4096.log 2>&1; echo "R trace rc=$?"
f=$(find $O/r4096 -name "*kernel_trace.csv" | head -1); python3 scripts/trace_window.py "$f" 300 k_contact_step_team
timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/c1" -o run --output-format csv -- python3 scripts/run_steps.py --config C1 --steps 300 > $O/c1.log 2>&1; echo "C1 trace rc=$?"
f=$(find $O/c1 -name "*kernel_trace.csv" | head -1); python3 scripts/trace_window.py "$f" 300 k_density_small
exit 0
