# Bit-identity of two library variants: per-step state hashes (tests/hash_run.py) of C3 for 60 steps and the slab
# dam-break for 300 steps under build/variants/lib_$1.so and lib_$2.so.
set +e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/hash
for v in $1 $2; do
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python tests/hash_run.py gpurun_out/hash/c3_$v.json 60 C3 || exit 1
  SPHHIP_LIB=build/variants/lib_$v.so timeout -k 10 200 python tests/hash_run.py gpurun_out/hash/slab_$v.json 300 slab || exit 1
done
python3 - "$1" "$2" <<'PY'
import json, sys
a, b = sys.argv[1], sys.argv[2]
for c in ("c3", "slab"):
    ha = json.load(open(f"gpurun_out/hash/{c}_{a}.json"))["hashes"]
    hb = json.load(open(f"gpurun_out/hash/{c}_{b}.json"))["hashes"]
    print(c, "steps", len(ha), "identical" if ha == hb else f"DIFFER from step {next(i for i, (x, y) in enumerate(zip(ha, hb)) if x != y)}")
PY
