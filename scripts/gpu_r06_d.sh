# r6 d: interleaved A/B of the re-sort at C3 (bench.py 200 steps from rest + 200 mid-collapse): head against r5's
# resort.hip in the current library (r5rs) and head with r5's 8,192-slot ranges (rk8k). build/variants/ from
# scripts/build_variant.sh.
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06d; mkdir -p $O; export TMPDIR=/tmp
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
bash scripts/variant_ab.sh "${AB_VARIANTS:-head r5rs rk8k}" 3 > $O/ab.log 2>&1; rc=$?
cat $O/ab.log
exit $rc
