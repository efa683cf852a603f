# Register / LDS / spill summary of every kernel in one csrc file (device-only compile, readelf notes).
# Usage: bash scripts/kernel_resources.sh field_step [regex]
set -o pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${TMPDIR:-/tmp}/nof_res_$1.co
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -DNOF_ABLATE=${NOF_ABLATE:-0} --offload-device-only -c \
    $R/bundlesdf_amd/csrc/$1.hip -o $OUT.bundle || exit 1
/opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input=$OUT.bundle \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output=$OUT || exit 1
/opt/rocm/lib/llvm/bin/llvm-readelf --notes $OUT | python3 -c "
import re, sys
txt = sys.stdin.read()
for blk in txt.split('- .agpr_count')[1:]:
    def g(k):
        m = re.search(r'\.' + k + r':\s+(\S+)', blk)
        return m.group(1) if m else '?'
    name = g('name')
    if re.search(sys.argv[1], name):
        print(f\"{name[:90]:90s} vgpr {g('vgpr_count'):>4} agpr {blk.split()[0]:>3} sgpr {g('sgpr_count'):>4} \"
              f\"spill {g('vgpr_spill_count')} lds {g('group_segment_fixed_size')}\")
" "${2:-.}"
