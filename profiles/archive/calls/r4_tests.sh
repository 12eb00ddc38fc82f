# the whole GPU test suite on the in-tree build, then smoke
set -u
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/r4/gputest.log 2>&1
rc=$?; echo "gpu tests rc=$rc"; tail -3 gpurun_out/r4/gputest.log; if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 gpurun_out/r4/smoke.log; exit $rc
