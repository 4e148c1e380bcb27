#!/bin/bash
# Round 6: counters of the C4 x 8 loopback's receipt-wave kernels by phase (bins: k_gs_bins_count /
# k_gs_bins_place / k_shard_unpack_bins; GP_LIB=lib_nobins: k_gs_full4x / k_shard_unpack).
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
P3="TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
export PMC_PASSES="$P1;$P2;$P3;FETCH_SIZE;WRITE_SIZE"
OUT=${OUT:-r6_bins_pmc} PMC_CMD="tools/shard_loopback_prof.py --world 8 --n 100000000 --topology full --algorithm gossip" \
  PMC_RK=k_gs_sparse_x,k_gs_bins_count,k_gs_full4x PMC_WORLD=8 PMC_WARMUP=9 PMC_LINES=80 \
  PMC_KERNELS=k_gs_bins_count,k_gs_bins_place,k_shard_unpack_bins,k_gs_full4x,k_shard_unpack,k_scan_apply,k_shard_done_out \
  bash tools/gpu.sh pmcphase
