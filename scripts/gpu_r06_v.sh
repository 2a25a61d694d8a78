# r6 v: 128-target workgroups for pass 1 (tt128), pass 2 (tf128) or both (b128) against head at C2 (1,024 workgroups
# of 256 on 256 CUs: one partial round) and C3; headline parity on each variant first (the sparse-path counts
# assume 256-target blocks, so that test is left out).
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06v; mkdir -p $O; export TMPDIR=/tmp
for v in head tt128 tf128 b128; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 300 python -u -m pytest -x -q -p no:cacheprovider --timeout 200 --timeout-method thread tests/test_gpu_parity_headline.py -k "not sparse_paths" > $O/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -20 $O/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 $O/pytest_$v.log)"
done
for r in 1 2; do for cfg in C2 C3; do for v in head tt128 tf128 b128; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python bench.py --config $cfg --no-cpu-baseline --steps 200 --mid-steps 200 --mid-at 3000 > $O/ab_${v}_$cfg.log 2>&1 || { echo "$v $cfg failed"; tail -3 $O/ab_${v}_$cfg.log; exit 1; }
  python3 - "$v" "$cfg" "$r" "$O" <<'PY'
import json, sys
v, cfg, r, O = sys.argv[1:]
d = json.loads(open(f"{O}/ab_{v}_{cfg}.log").read().strip().splitlines()[-1])
print(r, cfg, v, "ms", d["ms_per_step"], d["kernels_ms_per_step"], "mid", d.get("ms_per_step_mid_collapse"), d.get("kernels_ms_per_step_mid_collapse"), flush=True)
PY
done; done; done
