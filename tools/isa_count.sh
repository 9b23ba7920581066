#!/bin/bash
# Static instruction mix and register counts of kernels in the gfx950 ISA of one HIP source
# (CPU only).  usage: tools/isa_count.sh <file.hip> <kernel-symbol-regex>
set -e
SRC="$1"; PAT="$2"
DIR=$(cd "$(dirname "$0")/.." && pwd)
OUT=$(mktemp -d)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -std=c++17 -I"$DIR/include" \
  --offload-device-only -S -o "$OUT/k.s" "$SRC"
python3 - "$OUT/k.s" "$PAT" <<'EOF'
import re, sys
text = open(sys.argv[1]).read()
pat = re.compile(sys.argv[2])
for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)^\.Lfunc_end\d+:", text, re.S | re.M):
    name, body = m.group(1), m.group(2)
    if not pat.search(name):
        continue
    ins = [l.split()[0] for l in body.splitlines() if l.startswith("\t") and not l.lstrip().startswith((".", ";"))]
    valu = sum(i.startswith("v_") for i in ins)
    salu = sum(i.startswith("s_") for i in ins)
    vmem = sum(i.startswith(("global_", "buffer_", "flat_")) for i in ins)
    meta = {}
    for key in ("vgpr_count", "sgpr_count", "agpr_count"):
        g = re.search(r"\.name:\s+" + re.escape(name) + r"\n(?:.*\n)*?.*\." + key + r":\s+(\d+)", text)
        meta[key] = g.group(1) if g else "?"
    print(f"{name[:100]}\n    static VALU {valu}  SALU {salu}  VMEM {vmem}  "
          f"vgpr {meta['vgpr_count']}  agpr {meta['agpr_count']}  sgpr {meta['sgpr_count']}")
EOF
rm -rf "$OUT"
