# round 3: all GPU tests (incl. C4/C5 parity, chunked passes, multi-GPU checks), then an interleaved
# A/B of the pass chunking (SPH_CHUNKS 1 / 2 / 4 / 8), then the gloo rehearsal of bench's N>1 check
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q -p no:cacheprovider --timeout=600 --timeout-method thread -rA > gpurun_out/pytest_gpu.log 2>&1; rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|FAILED|error" gpurun_out/pytest_gpu.log | tail -12
[ $rc -gt 1 ] && exit $rc
for round in 1 2; do
  for c in 1 4 2 8; do
    SPH_CHUNKS=$c timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --mid-steps 200 > gpurun_out/chunks_$c.log 2>&1 || { echo "chunks $c failed"; tail -3 gpurun_out/chunks_$c.log; exit 1; }
    python3 - "$c" "$round" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/chunks_{sys.argv[1]}.log").read().strip().splitlines()[-1])
print(sys.argv[2], "chunks", sys.argv[1], "ms", d["ms_per_step"], d["kernels_ms_per_step"], "mid", d.get("ms_per_step_mid_collapse"), d.get("kernels_ms_per_step_mid_collapse"), flush=True)
PY
  done
done
SPH_DIST_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --transport python --steps 10 --warmup 2 > gpurun_out/bench_gloo2.log 2>&1; rc=$?
echo "gloo2 rc=$rc"; grep -E '^\{' gpurun_out/bench_gloo2.log | tail -c 2500
exit 0
