#!/bin/bash
# Build libgossip_hip.so (+ the CLI) of git revision REV into cop5615-gossip_protocol_amd/lib_NAME/ for a
# loopback or CLI A/B against the working tree (GP_LIB=lib_NAME).  The revision must share the working
# tree's ABI for the Python tools.   bash tools/variants/build_rev.sh HEAD pre
set -e
REV=$1; NAME=$2
R=$(cd "$(dirname "$0")/../.." && pwd); P=$R/cop5615-gossip_protocol_amd; T=$(mktemp -d)
mkdir -p $T/csrc $T/include $P/lib_$NAME
for f in gp_kernels.hip gp_api.cpp gp_kernels.h gp_common.h gossip_cli.cpp; do
  git -C $R show $REV:cop5615-gossip_protocol_amd/csrc/$f > $T/csrc/$f
done
git -C $R show $REV:include/gossip_hip.h > $T/include/gossip_hip.h
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -I$T/include -I$T/csrc \
  -shared -o $P/lib_$NAME/libgossip_hip.so $T/csrc/gp_kernels.hip $T/csrc/gp_api.cpp -ldl
/opt/rocm/bin/hipcc -O2 -std=c++17 -Wall -I$T/include -o $P/lib_$NAME/gossip $T/csrc/gossip_cli.cpp \
  -L$P/lib_$NAME -lgossip_hip -Wl,-rpath,'$ORIGIN'
rm -rf $T
