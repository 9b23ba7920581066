#!/bin/bash
# Timing-only diagnostic builds of the lean integrate kernel (MQR_DIAG in vbg_kernels.hpp):
#   1 = projection + update without the depth gathers, 2 = projection + gathers without the update;
#   tiled kernel (k_integrate_lt, variant 5): 3 = no LDS depth reads, 4 = no tile copies, 5 = neither.
# Their results are wrong by construction; they only locate where the kernel's time goes.
#   bash tools/diag_integrate.sh build          # here (CPU): tools/_diag/libmqr_diag{1,2}.so
#   bash tools/diag_integrate.sh run            # on the GPU box: ab_integrate.py against each build
set -o pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
CSRC="$ROOT/metaquest-3d-reconstruction_amd/csrc"
if [ "$1" = build ]; then
  mkdir -p "$ROOT/tools/_diag"
  make -C "$CSRC" >/dev/null || exit 1  # the other objects come from the regular build
  for d in ${DIAGS:-1 2}; do
    tmp=$(mktemp -d)
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -I"$ROOT/include" \
      -fno-slp-vectorize -DMQR_AB=1 -DMQR_DIAG=$d -c "$CSRC/vbg.hip" -o "$tmp/vbg.o" || exit 1
    objs=$(ls "$CSRC"/build/*.o | grep -v "/vbg.o$")
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$ROOT/tools/_diag/libmqr_diag$d.so" "$tmp/vbg.o" $objs \
      -Wl,-rpath,/opt/rocm/lib -ldl || exit 1
    rm -rf "$tmp"
  done
elif [ "$1" = run ]; then
  mkdir -p "$ROOT/gpurun_out"
  for d in ${DIAGS:-1 2}; do
    MQR_HIP_LIB="$ROOT/tools/_diag/libmqr_diag$d.so" timeout -k 10 300 python3 -u "$ROOT/tools/ab_integrate.py" \
      --variants "${VARIANTS:-0,3}" --rounds 5 > "$ROOT/gpurun_out/ab_diag$d.json" || exit 1
  done
else
  echo "usage: $0 build|run"; exit 2
fi
