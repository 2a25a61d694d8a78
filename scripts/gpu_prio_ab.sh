# A/B of the slab step's comm-stream knobs, serialised per-slab cost (scripts/slab_overhead.py) and N = 2 / 4 traces:
#   hi   SPH_COMM_PRIORITY=1 (default: the device's highest stream priority), folded early count (default)
#   lo   SPH_COMM_PRIORITY=0
#   nf   SPH_NO_FOLDED_COUNT=1 (the early sends' count as its own launch)
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/prio; export TMPDIR=/tmp
run_cfg() {
  case $1 in
    hi) env SPH_COMM_PRIORITY=1 "${@:2}" ;;
    lo) env SPH_COMM_PRIORITY=0 "${@:2}" ;;
    nf) env SPH_COMM_PRIORITY=1 SPH_NO_FOLDED_COUNT=1 "${@:2}" ;;
  esac
}
for round in 1 2; do
  for c in hi lo nf; do
    run_cfg $c timeout -k 10 300 python -u scripts/slab_overhead.py 2,4,8 100 --no-concurrent > gpurun_out/prio/ovh_${c}_$round.log 2>&1; rc=$?
    echo "$c round $round rc=$rc"; tail -3 gpurun_out/prio/ovh_${c}_$round.log | cut -c 1-260
    [ $rc -ne 0 ] && exit $rc
  done
done
for c in hi lo nf; do
  for n in 2 4; do
    SPH_COMM_PRIORITY=$([ $c = lo ] && echo 0 || echo 1) SPH_NO_FOLDED_COUNT=$([ $c = nf ] && echo 1 || echo) timeout -k 10 180 rocprofv3 --kernel-trace --stats -d "$GRAFT_REPO_ROOT/gpurun_out/prio/k${n}_$c" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/slab_trace.py" $n 40 > gpurun_out/prio/k${n}_$c.log 2>&1; rc=$?
    echo "trace $n $c rc=$rc"
    [ $rc -ne 0 ] && exit $rc
  done
done
exit 0
