# which k_simx switch the poisoned config3_epaxos failure follows
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/r5b; mkdir -p $M
for cfg in "FX_SIMX_PF=1" "FX_SIMX_PF=0" "FX_SIMX_LX=0"; do
  env $cfg timeout -k 10 300 python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu \
    "tests/test_poison_all.py::test_poisoned_k_simx" -k "config3" > $M/$cfg.log 2>&1
  echo "$cfg rc=$?: $(tail -1 $M/$cfg.log)"
done
