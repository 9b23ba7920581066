#!/bin/bash
# Libraries that differ only in the confidence object, for process-alternating A/B timing with
# tools/conf_workload.py (MQR_HIP_LIB=tools/_ab/libmqr_conf_<name>.so):
#   old  the committed confidence.hip of git revision $OLD_REV (default HEAD), product flags
#   new  the working-tree confidence.hip, product flags (-fno-slp-vectorize)
#   slp  the working-tree confidence.hip with SLP vectorisation
#   w8 / slpw8  new / slp with k_confidence held to 8 waves per SIMD (amdgpu_waves_per_eu(8, 8))
set -e
cd "$(dirname "$0")/../metaquest-3d-reconstruction_amd/csrc"
make -s build/vbg.o build/extract.o build/ingest.o
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -I../../include -I. -Wall -Wno-unused-result --offload-compress"
mkdir -p ../../tools/_ab build/var
git show ${OLD_REV:-HEAD}:metaquest-3d-reconstruction_amd/csrc/confidence.hip > build/var/confidence_old.hip
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DMQR_SRC_TAG=\"var-old\" -c build/var/confidence_old.hip -o build/var/c_old.o
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DMQR_SRC_TAG=\"var-new\" -c confidence.hip -o build/var/c_new.o
/opt/rocm/bin/hipcc $F -DMQR_SRC_TAG=\"var-slp\" -c confidence.hip -o build/var/c_slp.o
# (the working tree's kernel carries amdgpu_waves_per_eu(8, 8) since round 4: then w8 = new)
sed 's/__launch_bounds__(256) void k_confidence/__launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8, 8))) void k_confidence/' \
  confidence.hip > build/var/confidence_w8.hip
grep -q "amdgpu_waves_per_eu(8, 8))) void k_confidence" build/var/confidence_w8.hip
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DMQR_SRC_TAG=\"var-w8\" -c build/var/confidence_w8.hip -o build/var/c_w8.o
/opt/rocm/bin/hipcc $F -DMQR_SRC_TAG=\"var-slpw8\" -c build/var/confidence_w8.hip -o build/var/c_slpw8.o
for v in old new slp w8 slpw8; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_ab/libmqr_conf_$v.so \
    build/vbg.o build/extract.o build/ingest.o build/var/c_$v.o -Wl,-rpath,/opt/rocm/lib -ldl
done
