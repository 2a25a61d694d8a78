set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python bench.py --strong --config C4 --no-cpu-baseline --steps 100 --warmup 10 > gpurun_out/strong_C4.log 2>&1; echo "C4 rc=$?"; tail -1 gpurun_out/strong_C4.log | cut -c 1-400
timeout -k 10 300 python bench.py --strong --config C5 --no-cpu-baseline --steps 50 --warmup 5 > gpurun_out/strong_C5.log 2>&1; echo "C5 rc=$?"; tail -1 gpurun_out/strong_C5.log | cut -c 1-400
timeout -k 10 400 python -u scripts/long_run.py --config C3 --steps 20000 --every 1000 > gpurun_out/long_run.log 2>&1; echo "long rc=$?"; tail -5 gpurun_out/long_run.log
