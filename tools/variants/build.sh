# Build tuning variants of the kernel file into cop5615-gossip_protocol_amd/lib_<name>/ (GP_LIB selects one).
set -e
R=$(cd "$(dirname "$0")/../.." && pwd); P=$R/cop5615-gossip_protocol_amd
for f in "$@"; do
  n=$(basename $f .hip); mkdir -p $P/lib_$n
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -Wall -I$R/include -I$P/csrc -shared -o $P/lib_$n/libgossip_hip.so $f $P/csrc/gp_api.cpp &
done
wait
