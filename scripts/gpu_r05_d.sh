# Round 5: the reference's scale — small-N timing (Model R 4096 / 32768, C1) and kernel traces of R4096 and C1.
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05d; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1; echo "small-N rc=$?"; grep -v amdgpu.ids $O/small_n.log
timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/r4096" -o run --output-format csv -- python3 scripts/run_steps.py --model-r 4096 --steps 300 > $O/r4096.log 2>&1; echo "R trace rc=$?"
f=$(find $O/r4096 -name "*kernel_trace.csv" | head -1); python3 scripts/trace_window.py "$f" 300 k_contact_step_team
timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/$O/c1" -o run --output-format csv -- python3 scripts/run_steps.py --config C1 --steps 300 > $O/c1.log 2>&1; echo "C1 trace rc=$?"
f=$(find $O/c1 -name "*kernel_trace.csv" | head -1); python3 scripts/trace_window.py "$f" 300 k_density_small
exit 0
