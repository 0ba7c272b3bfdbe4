# VGPR / AGPR / spill counts of the quad kernels in a HIP object or shared
# library (dev aid): bash tools/kernel_regs.sh FILE [NAME_REGEX]
set -e
F=$1; RX=${2:-quad}
T=$(mktemp -d)
B=/opt/rocm/lib/llvm/bin
$B/llvm-objcopy --dump-section=.hip_fatbin=$T/fat.bin "$F" 2>/dev/null || cp "$F" $T/fat.bin
$B/clang-offload-bundler --unbundle --type=o --input=$T/fat.bin \
  --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$T/k.co
$B/llvm-readelf --notes $T/k.co > $T/notes.txt
python3 - "$T/notes.txt" "$RX" <<'PY'
import re, sys
t = open(sys.argv[1]).read()
for b in t.split('  - .agpr_count')[1:]:
    n = re.search(r'\.name:\s+(\S+)', b).group(1)
    if not re.search(sys.argv[2], n):
        continue
    g = lambda k: (re.search(r'\.%s:\s+(\d+)' % k, b) or [None, '?'])[1]
    print(f"{n[:70]:70s} vgpr {g('vgpr_count'):>4s} agpr {b.split(chr(10))[0].split(':')[-1].strip():>4s} "
          f"spill {g('vgpr_spill_count')} lds {g('group_segment_fixed_size')}")
PY
rm -rf $T
