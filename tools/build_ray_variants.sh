#!/bin/bash
# Libraries that differ only in the ray-casting object, for process-alternating A/B timing with
# tools/raycast_workload.py (MQR_HIP_LIB=tools/_ab/libmqr_ray_<name>.so): xcd = MQR_RAY_XCD=1, plain =
# MQR_RAY_XCD=0.  (Round 4 measured the XCD-banded order this way and removed it; the
# macro is gone from raycast.hip, so both builds are now the plain order -- edit raycast.hip to A/B.)
set -e
cd "$(dirname "$0")/../metaquest-3d-reconstruction_amd/csrc"
make -s $(for s in vbg extract confidence ingest meshfilter merge color; do echo build/$s.o; done)
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -I../../include -I. -Wall -Wno-unused-result --offload-compress"
mkdir -p ../../tools/_ab build/var
for v in xcd plain; do
  x=1; [ $v = plain ] && x=0
  /opt/rocm/bin/hipcc $F -DMQR_RAY_XCD=$x -c raycast.hip -o build/var/r_$v.o
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_ab/libmqr_ray_$v.so \
    build/vbg.o build/extract.o build/confidence.o build/ingest.o build/meshfilter.o build/merge.o build/color.o \
    build/var/r_$v.o -Wl,-rpath,/opt/rocm/lib -ldl
done
