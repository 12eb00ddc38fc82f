# .private_segment_fixed_size (scratch bytes per lane) of every kernel in one
# of the library's objects, from its gfx950 code object's metadata notes.
# usage: bash tools/scratch_check.sh fantoch_amd/build/obj/sim_big.hip.o [name filter]
set -e -o pipefail
B=/opt/rocm/lib/llvm/bin
T=$(mktemp -d)
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$1"
$B/clang-offload-bundler --type=o --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --input=$T/fat.bin --output=$T/k.co --unbundle
$B/llvm-readelf --notes $T/k.co | python3 -c "
import sys, re
flt = sys.argv[1] if len(sys.argv) > 1 else ''
name = priv = None
rows = []
for l in sys.stdin:
    m = re.match(r'\s+\.name:\s+(\S+)', l)
    if m: name = m.group(1)
    m = re.match(r'\s+\.private_segment_fixed_size:\s+(\d+)', l)
    if m: priv = int(m.group(1))
    if name and priv is not None and re.match(r'\s+\.(name|private_segment_fixed_size):', l):
        pass
    m = re.match(r'\s+\.vgpr_spill_count:\s+(\d+)', l)
    if m and name:
        rows.append((name, priv)); name = priv = None
for n, p in rows:
    if flt in n: print('%6s  %s' % (p, n))
" "${2:-}"
rm -rf $T
