#!/bin/bash
# Final round-4 run of the committed build (each step under its own limit, tools/gpu_steps.sh; stops at the first
# step that faults / times out): the GPU test suite and smoke, the driver-style bench line, a kernel trace of a bench
# run (serial schedule), the per-layer conv report, the PMC HBM traffic of one step (tools/pmc_run.sh), and the
# full-size C3-C5 steps with their HIP-graph replays.  Parse on the CPU afterwards (tools/prof_summary.py,
# tools/pmc_step.py --parse).
bash tools/gpu_steps.sh \
  "700 gputests python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "120 smoke python -c 'import __graft_entry__ as g; g.smoke()'" \
  "400 bench python bench.py" \
  "300 btrace env SSSEG_OVERLAP_TEACHER=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/btrace -o b -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-fp32 --no-graph" \
  "300 layers python tools/layer_report.py" \
  "600 pmc bash tools/pmc_run.sh" \
  "600 full python tools/full_size_steps.py --graph"
