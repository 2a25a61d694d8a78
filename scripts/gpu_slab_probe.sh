# Per-slab cost probe: serialised overhead at N = 2, 4, 8, and kernel traces of C3 on one context and of C3 x 2 / x 4
# serialised (scripts/slab_trace.py), for side-by-side kernel durations.
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/slabtrace; export TMPDIR=/tmp
timeout -k 10 300 python -u scripts/slab_overhead.py 2,4,8 100 --no-concurrent > gpurun_out/slab_overhead.log 2>&1; rc=$?
echo "slab_overhead rc=$rc"; tail -4 gpurun_out/slab_overhead.log
[ $rc -ne 0 ] && exit $rc
for n in 1 2 4; do
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/slabtrace/k$n" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/slab_trace.py" $n 40 > gpurun_out/slabtrace/k$n.log 2>&1; rc=$?
  echo "trace $n rc=$rc"; tail -1 gpurun_out/slabtrace/k$n.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
