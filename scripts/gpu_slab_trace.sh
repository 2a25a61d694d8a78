set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/slabtrace; export TMPDIR=/tmp
for n in 1 4; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/slabtrace/k$n" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/slab_trace.py" $n 30 > gpurun_out/slabtrace/k$n.log 2>&1; rc=$?
  echo "kernel trace n=$n rc=$rc"; tail -1 gpurun_out/slabtrace/k$n.log
  [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 180 rocprofv3 --kernel-trace --hip-runtime-trace -d "$GRAFT_REPO_ROOT/gpurun_out/slabtrace/h4" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/slab_trace.py" 4 30 > gpurun_out/slabtrace/h4.log 2>&1; rc=$?
echo "hip trace rc=$rc"; tail -1 gpurun_out/slabtrace/h4.log
exit 0
