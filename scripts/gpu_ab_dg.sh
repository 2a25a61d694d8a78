# Density plane budget A/B, then the kernel trace of the mid-collapse section (per-kernel means).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/variant_ab.sh "head dg1500" 3 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/profmid" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --mid-steps 200 --no-cpu-baseline > gpurun_out/profmid.log 2>&1 || { echo "rocprof failed"; tail -5 gpurun_out/profmid.log; exit 1; }
python3 scripts/trace_kstats.py gpurun_out/profmid/run_kernel_trace.csv 1000 | tee gpurun_out/mid_kstats.txt
