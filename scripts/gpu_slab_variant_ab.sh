# Interleaved A/B of library variants on the slab step's serialised per-slab cost (scripts/slab_overhead.py), with
# the group bit-identity tests first on every variant:  bash scripts/gpu_slab_variant_ab.sh "head v1 v2" [rounds]
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/slab_ab; export TMPDIR=/tmp
for v in $1; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_multi.py -m gpu -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "bitwise or matches_single or collapse or early_sends" > gpurun_out/slab_ab/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -20 gpurun_out/slab_ab/pytest_$v.log; exit 1; }
  echo "$v: $(tail -1 gpurun_out/slab_ab/pytest_$v.log)"
done
for round in $(seq 1 ${2:-2}); do
  for v in $1; do
    SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 300 python -u scripts/slab_overhead.py 2,4,8 100 --no-concurrent > gpurun_out/slab_ab/ovh_${v}_$round.log 2>&1 || { echo "$v failed"; tail -5 gpurun_out/slab_ab/ovh_${v}_$round.log; exit 1; }
    python3 - "$v" "$round" <<'PY'
import ast, sys
v, r = sys.argv[1], sys.argv[2]
rows = [ast.literal_eval(l) for l in open(f"gpurun_out/slab_ab/ovh_{v}_{r}.log") if l.startswith("{'world'")]
print(r, v, " ".join(f"N={d['world']}: +{1e3 * d['overhead_per_slab_ms']:.1f}us" for d in rows), flush=True)
PY
  done
done
