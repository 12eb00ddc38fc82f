set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
bash tools/mode_pmc.sh dense "k_graph_wide<false" || exit 1
python3 tools/mode_pmc_summary.py dense gpurun_out/pmc_dense "k_graph_wide<false" profiles/r04f_ > gpurun_out/dense_summary.log 2>&1 || { tail -5 gpurun_out/dense_summary.log; exit 1; }
cp gpurun_out/pmc_dense/trace/*kernel_stats.csv profiles/r04f_dense_kernel_stats.csv
timeout -k 10 600 python3 bench.py --mode dense > gpurun_out/dense_bench.log 2>&1 || { tail -5 gpurun_out/dense_bench.log; exit 1; }
tail -1 gpurun_out/dense_bench.log | cut -c1-400
