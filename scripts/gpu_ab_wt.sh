# Write-through / non-temporal bulk-output stores vs plain stores: interleaved A/B, then the
# inter-kernel gaps of each build from a kernel trace.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
bash scripts/variant_ab.sh "head wt16 wt2" 3 || exit 1
export TMPDIR=/tmp
for v in head wt16 wt2; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 rocprofv3 --kernel-trace -d "$GRAFT_REPO_ROOT/gpurun_out/tr_$v" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/bench.py" --gpus 1 --steps 20 --warmup 5 --mid-steps 0 --no-cpu-baseline > gpurun_out/tr_$v.log 2>&1 || { echo "trace $v failed"; tail -5 gpurun_out/tr_$v.log; exit 1; }
  echo "== $v"; python3 scripts/trace_gaps.py gpurun_out/tr_$v/run_kernel_trace.csv 100 | head -5
done
