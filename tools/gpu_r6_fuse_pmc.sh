#!/bin/bash
# Round 6: counters of the 100M / 8 push-sum loopback's rank kernels by phase (HEAD: the dense round
# kernel routes its link messages; no k_ps_link_scatter_x): HBM bytes, texture-path busy, waves.
export PMC_PASSES="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS TA_TA_BUSY_sum TD_TD_BUSY_sum"
OUT=${OUT:-r6_fuse_pmc} PMC_CMD="tools/shard_loopback_prof.py --world 8 --n 100000000 --topology Imp3D --algorithm push-sum" \
  PMC_RK=k_ps_quiet_x PMC_WORLD=8 PMC_WARMUP=8 PMC_LINES=80 PMC_TIMEOUT=240 \
  PMC_KERNELS="k_ps_quiet_x<false>,k_ps_quiet_x<true>,k_shard_unpack,k_shard_halo,k_shard_pack" \
  bash tools/gpu.sh pmcphase
