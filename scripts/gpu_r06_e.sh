# r6 e: the re-sort with one share form per kernel instantiation (k_mv_rank<STAGED>): re-sort and path-independence
# tests on the in-tree library, then an interleaved C3 A/B: head2 (this) against head (both share forms in one
# kernel) and r5's resort.hip (r5rs).
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06e; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest tests/test_gpu_resort.py tests/test_gpu_path_independence.py -m gpu -v -s -p no:cacheprovider --timeout=300 --timeout-method thread -x > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error|'shape'|_resort" $O/pytest.log | tail -6
[ $rc -ne 0 ] && exit $rc
bash scripts/variant_ab.sh "${AB_VARIANTS:-head2 head r5rs}" 3 > $O/ab.log 2>&1; rc=$?
cat $O/ab.log
exit $rc
