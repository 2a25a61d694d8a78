# What the per-kernel HIP events cost the timed step: bench with and without the event pass, interleaved.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for r in 1 2 3; do
  for f in "" "--no-profile"; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 200 --mid-steps 0 $f > gpurun_out/pc.log 2>&1 || { tail -3 gpurun_out/pc.log; exit 1; }
    python3 -c "import json,sys; d=json.loads(open('gpurun_out/pc.log').read().strip().splitlines()[-1]); print(sys.argv[1], sys.argv[2] or 'profile', d['ms_per_step'], d.get('kernels_ms_per_step'))" "$r" "$f"
  done
done
