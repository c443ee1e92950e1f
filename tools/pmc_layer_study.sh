set -e
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM"
P2="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES GRBM_GUI_ACTIVE"
A3="--kind fwd --cin 384 --cout 128 --k 3 --hw 128 --batch 16"
A1="--kind fwd --cin 256 --cout 1024 --k 1 --hw 32 --batch 16"
bash tools/pmc_layer.sh gpurun_out/pmcl_a3 "$P1" "$A3" 14 3 6 8 19 21
bash tools/pmc_layer.sh gpurun_out/pmcl_b3 "$P2" "$A3" 14 3 6 8 19 21
bash tools/pmc_layer.sh gpurun_out/pmcl_a1 "$P1" "$A1" 20 15 22 3
bash tools/pmc_layer.sh gpurun_out/pmcl_b1 "$P2" "$A1" 20 15 22 3
