# the drop-in handle's bench line (a latency metric: no HBM roofline)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
P=${PREFIX:-gpurun_out/r5prof/r05a_}
mkdir -p $(dirname $P)
timeout -k 10 300 python3 bench.py --mode handle > gpurun_out/r5m_handle.log 2>&1 || { echo "handle rc=$?"; tail -5 gpurun_out/r5m_handle.log; exit 1; }
tail -1 gpurun_out/r5m_handle.log > ${P}handle_bench.json
cut -c1-300 ${P}handle_bench.json
