# PMC comparison of library builds (profiling only): for each library path (relative to the repo
# root), one rocprofv3 --pmc pass per counter group on a C3 stepping run; summarised per kernel.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/pmcl
export TMPDIR=/tmp
i=0
for lib in "$@"; do
  i=$((i+1)); g=0
  for grp in "SQ_INSTS_VALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_WAIT_INST_LDS" "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    g=$((g+1))
    SPHHIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $grp -d "$GRAFT_REPO_ROOT/gpurun_out/pmcl/l${i}_g$g" -o run --output-format csv -- python3 "$GRAFT_REPO_ROOT/scripts/run_steps.py" --config C3 --steps 10 --warmup 2 > gpurun_out/pmcl/l${i}_g$g.log 2>&1
  done
  echo "lib $i = $lib"
done
python3 - "$@" <<'PY'
import csv, glob, os, re, sys
from collections import defaultdict
for i, lib in enumerate(sys.argv[1:], 1):
    acc = defaultdict(lambda: defaultdict(list))
    for d in glob.glob(f"gpurun_out/pmcl/l{i}_g*"):
        f = os.path.join(d, "run_counter_collection.csv")
        if not os.path.exists(f):
            continue
        for r in csv.DictReader(open(f)):
            k = re.sub(r"<[^>]*>$", "", r["Kernel_Name"].split("(")[0].replace("void ", "").replace("sph::", ""))
            if k in ("k_force_tiled", "k_density_tiled"):
                acc[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        out = {c: round(v / 1e6, 2) for c, v in sorted(m.items())}
        if "FETCH_SIZE" in m and "WRITE_SIZE" in m:
            out["hbm_MB"] = round((2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024 / 1e6, 1)
        if m.get("SQ_LDS_IDX_ACTIVE"):
            out["lds_conflict_share"] = round(m["SQ_LDS_BANK_CONFLICT"] / m["SQ_LDS_IDX_ACTIVE"], 3)
        if "TCC_HIT_sum" in m:
            out["tcc_hit"] = round(m["TCC_HIT_sum"] / max(1.0, m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 3)
        print(lib, k, out)
PY
