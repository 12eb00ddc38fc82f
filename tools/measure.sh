# Round measurement: HBM traffic PMC passes + kernel-trace stats of the default bench.
# usage: bash tools/measure.sh [extra bench args]; outputs under gpurun_out/meas/
set -e
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
M=gpurun_out/meas; rm -rf $M; mkdir -p $M
B="bench.py --steps 1 --warmup 1 --no-cpu-baseline $*"
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE -d $M/fetch -o pmc --output-format csv -- python3 $B > $M/fetch.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d $M/write -o pmc --output-format csv -- python3 $B > $M/write.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $M/trace -o run --output-format csv -- python3 bench.py $* > $M/bench.log 2>&1
tail -1 $M/bench.log
find $M -name "*stats*"
