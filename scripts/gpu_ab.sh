# A/B alternate builds of libsphhip.so (profiling only): for each library path given
# (relative to the repo root), time the neighbour passes with scripts/nb_variants.py.
set -e
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
V=${AB_VARIANTS:-1}
for lib in "$@"; do
  echo "== $lib"
  SPHHIP_LIB=$GRAFT_REPO_ROOT/$lib timeout -k 10 300 python3 scripts/nb_variants.py --variants $V --steps 20 --rounds ${AB_ROUNDS:-3}
done
