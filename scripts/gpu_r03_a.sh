# round 3 first pass: GPU tests (new C4/C5 parity, multi-GPU checks), bench line, gloo rehearsal of the N>1 check
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout=600 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|error" gpurun_out/pytest_gpu.log | tail -5
[ $rc -gt 1 ] && exit $rc
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --mid-steps 0 --no-cpu-baseline > gpurun_out/bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -c 3000 gpurun_out/bench.log
[ $rc -ne 0 ] && exit $rc
SPH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --transport python --steps 10 --warmup 2 > gpurun_out/bench_gloo2.log 2>&1; rc=$?
echo "gloo2 rc=$rc"; grep -E '^\{' gpurun_out/bench_gloo2.log | tail -c 2500
exit 0
