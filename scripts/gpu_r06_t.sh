# r6 t: isolating r6 s's changes on one box: head (the DPP-scan commit), new (all of r6 s), noscan (r6 s without the
# stayer-rank scan table), nosel (r6 s without the select chains); small-N rates, two rounds.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06t; mkdir -p $O; export TMPDIR=/tmp
for r in 1 2; do for v in head new noscan nosel; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python -u scripts/small_n_timing.py 500 > $O/small_n_${v}_$r.log 2>&1; rc=$?
  echo "== $v $r rc=$rc"; grep -E "sphere N=4096 team default|C1" $O/small_n_${v}_$r.log | cut -c 1-110; [ $rc -ne 0 ] && exit $rc
done; done
exit 0
