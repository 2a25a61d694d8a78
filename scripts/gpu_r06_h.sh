# r6 h: the Model R one-launch step's phase clocks at the final head (probe build), and the splash state's GPU step
# dumped for the pass-2 margin analysis on the CPU (scripts/pass2_margin.py).
set +e
cd "$GRAFT_REPO_ROOT"; O=gpurun_out/r06h; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 200 python -u scripts/contact_probe.py --steps 30 > $O/contact_probe.log 2>&1; rc=$?
echo "probe rc=$rc"; tail -2 $O/contact_probe.log; [ $rc -ne 0 ] && exit $rc
timeout -k 10 200 python -u scripts/contact_probe.py --steps 30 --n 32768 > $O/contact_probe_32k.log 2>&1; rc=$?
echo "probe 32k rc=$rc"; tail -2 $O/contact_probe_32k.log
timeout -k 10 200 python -u scripts/splash_dump.py --out $O/splash_gpu.npz > $O/splash_dump.log 2>&1; rc=$?
echo "dump rc=$rc"; tail -2 $O/splash_dump.log
exit $rc
