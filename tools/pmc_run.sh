#!/bin/bash
# One C2 training step under rocprofv3: FETCH_SIZE and WRITE_SIZE in separate --pmc passes (the TCC block cannot
# hold both), then a kernel trace of the same step; parse on the CPU with
#   python tools/pmc_step.py --parse gpurun_out/pmc_f gpurun_out/pmc_w --trace gpurun_out/pmc_t > profiles/<name>.json
#   python tools/pmc_step.py --mfma gpurun_out/pmc_m --trace gpurun_out/pmc_t > profiles/<name>_mfma.json
# (the MFMA pass: SQ_VALU_MFMA_BUSY_CYCLES, SQ_BUSY_CYCLES, GRBM_GUI_ACTIVE -- 2 SQ + 1 GRBM counters, one pass)
set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
rm -rf gpurun_out/pmc_f gpurun_out/pmc_w gpurun_out/pmc_m gpurun_out/pmc_t
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o f --output-format csv -- python tools/pmc_step.py > gpurun_out/pmc_f.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o w --output-format csv -- python tools/pmc_step.py > gpurun_out/pmc_w.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d gpurun_out/pmc_m -o m --output-format csv -- python tools/pmc_step.py > gpurun_out/pmc_m.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace -d gpurun_out/pmc_t -o t --output-format csv -- python tools/pmc_step.py > gpurun_out/pmc_t.log 2>&1
