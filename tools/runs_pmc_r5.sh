P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
P2="SQ_WAVES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_SALU TA_TA_BUSY_sum TD_TD_BUSY_sum GRBM_GUI_ACTIVE"
P3="TCC_EA0_ATOMIC_sum TCC_ATOMIC_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"
export PMC_PASSES="$P1;$P2;$P3;FETCH_SIZE;WRITE_SIZE"
OUT=pmc_c4loop PMC_CMD="tools/shard_loopback_prof.py --world 8 --n 100000000 --topology full --algorithm gossip" PMC_RK=k_gs_full4x PMC_WORLD=8 PMC_WARMUP=8 PMC_KERNELS=k_gs_full4x,k_shard_unpack,k_shard_done_out,k_shard_pack bash tools/gpu.sh pmcphase && \
OUT=pmc_c4one PMC_CMD="tools/prof_run.py --n 100000000 --topology full --algorithm gossip --rounds 1000000" PMC_RK=k_gs_full4 PMC_WORLD=1 PMC_WARMUP=0 PMC_KERNELS=k_gs_full4,k_tally_rows,k_gs_tally_scatter_lds,k_gs_tally_count bash tools/gpu.sh pmcphase && \
OUT=pmc_c3 PMC_CMD="tools/prof_run.py --rounds 1000000" PMC_RK="k_ps_quiet<1>" PMC_WORLD=1 PMC_WARMUP=0 PMC_KERNELS="k_ps_quiet<1>" bash tools/gpu.sh pmcphase
