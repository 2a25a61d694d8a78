# N=1: single context vs the in-library decomposed step (RCCL communicator of one rank), C3, interleaved,
# with the bench's default sampled kernel timing; then the strong-scaling C4 line on one GPU.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2; do
  for f in "" "--slab"; do
    timeout -k 10 300 python bench.py --no-cpu-baseline --steps 200 --mid-steps 0 $f > gpurun_out/sl.log 2>&1 || { tail -5 gpurun_out/sl.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/sl.log').read().strip().splitlines()[-1]); print(sys.argv[1], sys.argv[2] or 'single', d['ms_per_step'], d['value'], d['config'].get('transport'), d.get('kernels_ms_per_step'))" "$r" "$f"
  done
done
timeout -k 10 300 python bench.py --no-cpu-baseline --strong --config C4 --steps 50 --mid-steps 0 > gpurun_out/strong_c4.log 2>&1 || { tail -5 gpurun_out/strong_c4.log; exit 1; }
tail -1 gpurun_out/strong_c4.log | cut -c1-400
