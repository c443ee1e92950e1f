#!/bin/bash
# Round-6 PMC study of the small-map ResNet layers the r5 verdict names (layer3 @16x32^2): per layer, three rocprofv3
# --pmc passes (wave-cycle anatomy, texture path / L2 latency, L2 hits / LDS conflicts) over tools/one_layer.py with the
# autotuned variant.  Parse: python tools/pmc_kernel.py gpurun_out/pmcl6_<layer>_<pass> igemm_glds
set -e
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_INST_LEVEL_VMEM SQ_INSTS_VMEM"
P2="TA_TA_BUSY TA_ADDR_STALLED_BY_TC_CYCLES TD_TD_BUSY TD_TC_STALL TCP_TCC_READ_REQ_LATENCY TCP_TCC_READ_REQ TCP_PENDING_STALL_CYCLES TCP_TCR_TCP_STALL_CYCLES GRBM_GUI_ACTIVE"
P3="TCC_HIT_sum TCC_MISS_sum SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
run() {   # name args
  local name=$1; shift
  for p in 1 2 3; do
    eval "c=\$P$p"
    timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/pmcl6_${name}_p$p -o p --output-format csv -- \
      python tools/one_layer.py "$@" --reps 5 > gpurun_out/pmcl6_${name}_p$p.log 2>&1
    tail -n 1 gpurun_out/pmcl6_${name}_p$p.log
  done
}
run k3fwd --kind fwd --cin 256 --cout 256 --k 3 --hw 32 --batch 16
run k3dgrad --kind dgrad --cin 256 --cout 256 --k 3 --hw 32 --batch 16
run k1fwd --kind fwd --cin 256 --cout 1024 --k 1 --hw 32 --batch 16
run k1dgrad --kind dgrad --cin 256 --cout 1024 --k 1 --hw 32 --batch 16
