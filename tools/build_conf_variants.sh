#!/bin/bash
# Libraries that differ only in the confidence object, for process-alternating A/B timing with
# tools/conf_workload.py (MQR_HIP_LIB=tools/_ab/libmqr_conf_<name>.so):
#   old  the committed confidence.hip of git revision $OLD_REV (default HEAD), product flags
#   new  the working-tree confidence.hip, product flags (-fno-slp-vectorize)
#   slp  the working-tree confidence.hip with SLP vectorisation
#   (w8 / slpw8, new / slp held to 8 waves per SIMD, measured in round 4: the production instances now
#   carry that attribute themselves)
#   xcd  new with the XCD-banded tile order (MQR_CONF_XCD=1, the default since round 4), plain: =0
#   (nt, the reference depth read and the outputs non-temporal, was measured in round 4 at -0.5 %,
#   within run-to-run spread, and not kept: r04v in profiles/r04_ab_confidence_variants.json)
set -e
cd "$(dirname "$0")/../metaquest-3d-reconstruction_amd/csrc"
make -s build/vbg.o build/extract.o build/ingest.o
F="--offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 -I../../include -I. -Wall -Wno-unused-result --offload-compress"
mkdir -p ../../tools/_ab build/var
git show ${OLD_REV:-HEAD}:metaquest-3d-reconstruction_amd/csrc/confidence.hip > build/var/confidence_old.hip
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DMQR_SRC_TAG=\"var-old\" -c build/var/confidence_old.hip -o build/var/c_old.o
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DMQR_SRC_TAG=\"var-new\" -c confidence.hip -o build/var/c_new.o
/opt/rocm/bin/hipcc $F -DMQR_SRC_TAG=\"var-slp\" -c confidence.hip -o build/var/c_slp.o
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DMQR_CONF_XCD=1 -DMQR_SRC_TAG=\"var-xcd\" -c confidence.hip -o build/var/c_xcd.o
/opt/rocm/bin/hipcc $F -fno-slp-vectorize -DMQR_CONF_XCD=0 -DMQR_SRC_TAG=\"var-plain\" -c confidence.hip -o build/var/c_plain.o
for v in old new slp xcd plain; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../../tools/_ab/libmqr_conf_$v.so \
    build/vbg.o build/extract.o build/ingest.o build/var/c_$v.o -Wl,-rpath,/opt/rocm/lib -ldl
done
