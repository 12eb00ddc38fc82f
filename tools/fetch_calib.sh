# FETCH_SIZE / WRITE_SIZE calibration for 4 B and 16 B per lane (tools/fetch_calib.hip):
# bash tools/fetch_calib.sh; output under gpurun_out/calib/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
M=gpurun_out/calib; rm -rf $M; mkdir -p $M
for c in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $c -d $M/$c -o pmc --output-format csv -- ./tools/build/fetch_calib \
    > $M/$c.log 2>&1 || { echo "$c rc=$?"; tail -5 $M/$c.log; exit 1; }
done
python3 - <<'PY'
import csv, glob
known = {"k_read4": 1 << 30, "k_read16": 1 << 30, "k_write4": 1 << 28}
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob("gpurun_out/calib/%s/**/*counter_collection.csv" % c, recursive=True):
        for r in csv.DictReader(open(f)):
            k = r["Kernel_Name"].split("(")[0].split()[-1]
            if r["Counter_Name"] == c and k in known:
                kb = float(r["Counter_Value"])
                print("%-9s %-10s %10.0f KB  = %.3f x the %d bytes touched" % (k, c, kb, kb * 1024 / known[k], known[k]))
PY
