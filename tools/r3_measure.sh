#!/bin/bash
# Round-3 measurement bundle: layer / vcat GPU tests, a tune-logged bench, and the PMC layer anatomy of the two
# representative 3x3 layers (tools/pmc_layer.sh) -- each step under its own limit (tools/gpu_steps.sh).
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM"
P2="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES GRBM_GUI_ACTIVE"
A3="--kind fwd --cin 384 --cout 128 --k 3 --hw 128 --batch 16"
A4="--kind fwd --cin 128 --cout 64 --k 3 --hw 256 --batch 16"
bash tools/gpu_steps.sh \
  "300 layertests python -u -m pytest tests/test_hip_layers.py tests/test_vcat.py -x -q --timeout 120 --timeout-method thread" \
  "200 tunelog env SSSEG_TUNE_LOG=1 python bench.py --steps 20 --no-cpu-baseline --no-fp32" \
  "200 pmc3 bash tools/pmc_layer.sh gpurun_out/pmcl_b3n \"$P2\" \"$A3\" 14 19 6 21" \
  "200 pmc4 bash tools/pmc_layer.sh gpurun_out/pmcl_b4n \"$P2\" \"$A4\" 15 20 14 1"
