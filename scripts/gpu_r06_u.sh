# r6 u: C2 (262,144 particles, one GPU) per-kernel breakdown: bench's HIP-event kernels and a rocprofv3 kernel trace,
# to see where C2 loses per-particle efficiency against C3 (rate table 2.20e9 against 3.25e9 particle-steps/s).
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06u; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --config C2 --no-cpu-baseline --steps 400 --mid-steps 400 --mid-at 3000 > $O/bench_C2.log 2>&1 &&
  tail -1 $O/bench_C2.log | cut -c 1-900 &&
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o c2 -- python bench.py --config C2 --no-cpu-baseline --no-profile --steps 200 --mid-steps 0 > $O/prof_C2.log 2>&1 &&
  find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/c2_kernel_stats.csv \; && cut -d, -f1-7 $O/c2_kernel_stats.csv | cut -c 1-60,200-400 | head -12
