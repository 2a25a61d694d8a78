# Force-pass ablation (profiling only): time k_force_tiled with the pair body stubbed (1),
# hits dropped after the scan (2), staging only (3), against the product build (0).
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for a in 1 2 3; do
  echo "== ablation $a"
  SPHHIP_LIB=$GRAFT_REPO_ROOT/sph-test_amd/build/abl$a/libsphhip.so timeout -k 10 300 python3 scripts/nb_variants.py --variants 1 --steps 5 --rounds 3
done
echo "== product"
timeout -k 10 300 python3 scripts/nb_variants.py --variants 1 --steps 5 --rounds 3
