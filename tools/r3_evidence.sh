#!/bin/bash
# End-of-round evidence bundle for the current build (each step under its own limit, tools/gpu_steps.sh):
# the driver-style bench line, a kernel trace of a bench run, the per-layer conv report, the PMC HBM traffic of one
# step (tools/pmc_run.sh: FETCH_SIZE / WRITE_SIZE passes + trace), and the full-size C3-C5 steps with their conv
# rooflines.  Parse on the CPU afterwards (tools/prof_summary.py, tools/pmc_step.py --parse).
bash tools/gpu_steps.sh \
  "400 bench python bench.py" \
  "300 btrace rocprofv3 --kernel-trace --output-format csv -d gpurun_out/btrace -o b -- python bench.py --steps 20 --no-cpu-baseline --no-fp32" \
  "300 layers python tools/layer_report.py" \
  "600 pmc bash tools/pmc_run.sh" \
  "600 full python tools/full_size_steps.py --layers"
