# r6 g (evidence at the final head): the Model R cell-skipping edge-state tests, the 2/4/8-rank RCCL rehearsal on one GPU (bench.py's slab check over RCCL must be
# bitwise against one context), and a 20,000-step C3 run (per-kernel means per 1,000-step window through the collapse).
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06g; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -k "cell_skipping" -m gpu -v -p no:cacheprovider --timeout=200 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|Error" $O/pytest.log | tail -5; [ $rc -ne 0 ] && exit $rc
RANKS="2 4 8" STEPS=60 WARMUP=10 LIMIT=300 bash scripts/gpu_rccl_rehearsal.sh > $O/rehearsal.log 2>&1; rc=$?
cat $O/rehearsal.log | cut -c 1-300; [ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u scripts/long_run.py --config C3 --steps 20000 --every 1000 > $O/long_run_C3.log 2>&1; rc=$?
tail -3 $O/long_run_C3.log | cut -c 1-200
exit $rc
