#!/bin/bash
# Kernel resource usage (VGPR/SGPR/spills/LDS) of the gfx950 code object in a
# built library: tools/kres.sh <lib.so> [kernel-name-regex]
set -eo pipefail
T=$(mktemp -d)
objcopy -O binary --only-section=.hip_fatbin "$1" "$T/fb.bin"
# one offload bundle per translation unit: split at the bundle magic
python3 - "$T" <<'PY'
import sys
d = sys.argv[1]
b = open(d + "/fb.bin", "rb").read()
mag = b"__CLANG_OFFLOAD_BUNDLE__"
pos = [i for i in range(len(b)) if b.startswith(mag, i)]
for k, i in enumerate(pos):
    open("%s/fb%d.bin" % (d, k), "wb").write(b[i:pos[k + 1] if k + 1 < len(pos) else len(b)])
PY
for f in "$T"/fb[0-9]*.bin; do
  /opt/rocm/lib/llvm/bin/clang-offload-bundler --unbundle --type=o --input="$f" \
    --targets=hipv4-amdgcn-amd-amdhsa--gfx950 --output="${f%.bin}.co"
done
for f in "$T"/fb[0-9]*.co; do /opt/rocm/lib/llvm/bin/llvm-readelf --notes "$f"; done | python3 -c '
import re, sys, subprocess
pat = re.compile(sys.argv[1] if len(sys.argv) > 1 else ".")
cur = {}
out = []
for line in sys.stdin:
    m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
    if not m: continue
    k, v = m.groups()
    if k == "agpr_count" and cur: out.append(cur); cur = {}
    cur[k] = v
out.append(cur)
for c in out:
    n = c.get("name", "")
    if not pat.search(n): continue
    dn = subprocess.run(["c++filt", n], capture_output=True, text=True).stdout.strip()
    dn = re.sub(r"std::conditional<[^>]*>::type", "T", dn)[:110]
    g = lambda k: str(c.get(k, "-"))
    print("vgpr %4s spill %3s sgpr %3s lds %6s scratch %5s  %s" % (g("vgpr_count"), g("vgpr_spill_count"),
          g("sgpr_count"), g("group_segment_fixed_size"), g("private_segment_fixed_size"), dn))
' "${2:-.}"
rm -rf "$T"
