# Random-atomic rates by footprint: u32 receipts vs u8 counters packed 4 per word
# (tools/microbench/atomics.hip).
set -o pipefail
mkdir -p gpurun_out/atomics
timeout -k 10 300 tools/microbench/atomics > gpurun_out/atomics/atomics.txt 2>&1; rc=$?; cat gpurun_out/atomics/atomics.txt; exit $rc
