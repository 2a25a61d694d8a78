# Companion measurements of the headline (round logs under profiles/): a 20,000-step C3 run through the
# collapse and the surge, BASELINE's C4 / C5 on one GPU through the decomposed step, and the --table rates.
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u scripts/long_run.py --config C3 --steps 20000 --every 1000 > gpurun_out/long_run.log 2>&1; rc=$?
echo "long_run rc=$rc"; tail -2 gpurun_out/long_run.log | cut -c 1-200; [ $rc -ne 0 ] && exit $rc
for c in C4 C5; do
  timeout -k 10 400 python bench.py --strong --config $c --steps 100 --warmup 10 --no-cpu-baseline > gpurun_out/strong_$c.log 2>&1; rc=$?
  echo "strong $c rc=$rc"; tail -1 gpurun_out/strong_$c.log | cut -c 1-300; [ $rc -ne 0 ] && exit $rc
done
timeout -k 10 600 python bench.py --table > gpurun_out/rate_table.log 2>&1; rc=$?
echo "table rc=$rc"; tail -6 gpurun_out/rate_table.log | cut -c 1-200
exit $rc
