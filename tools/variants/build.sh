# Build tuning variants of libgossip_hip.so into cop5615-gossip_protocol_amd/lib_<name>/ (GP_LIB=lib_<name>
# selects one).  Each argument is NAME:FLAGS, e.g.  k1:-DGP_TILE_K=1  (FLAGS: extra hipcc defines).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd); P=$R/cop5615-gossip_protocol_amd
for spec in "$@"; do
  n=${spec%%:*}; f=${spec#*:}; mkdir -p $P/lib_$n
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall $f -I$R/include -I$P/csrc \
    -shared -o $P/lib_$n/libgossip_hip.so $P/csrc/gp_kernels.hip $P/csrc/gp_api.cpp -ldl && \
  /opt/rocm/bin/hipcc -O2 -std=c++17 -Wall -I$R/include -o $P/lib_$n/gossip $P/csrc/gossip_cli.cpp \
    -L$P/lib_$n -lgossip_hip -Wl,-rpath,'$ORIGIN' &
done
wait
