# Model R pair body once per pair (the reaction torque from the same evaluation) and the chunk skip: bit-exact tests,
# small-N timing, PMC of the one-launch step.
set -u
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r05f; mkdir -p $O
( while true; do date >> $O/heartbeat; sleep 50; done ) & HB=$!
trap "kill $HB" EXIT
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  tests/test_gpu_fused.py tests/test_gpu_adhesion.py tests/test_gpu_contact_team.py tests/test_gpu_shipped_bonds.py \
  tests/test_gpu_path_independence.py tests/test_gpu_small.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 300 python -u scripts/small_n_timing.py 500 > $O/small_n.log 2>&1 || { tail -5 $O/small_n.log; exit 1; }
grep case $O/small_n.log
bash scripts/gpu_pmc_contact.sh > $O/pmc.log 2>&1 || { tail -5 $O/pmc.log; exit 1; }
tail -2 $O/pmc.log | cut -c1-900
