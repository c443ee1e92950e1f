#!/bin/bash
# Round-5 evidence of the committed build, in parts that each fit one gpurun call (tools/gpu_steps.sh: every step under
# its own limit, stop at the first fault / time limit).  Parse on the CPU afterwards: tools/trace_kernels.py and
# tools/prof_summary.py (kernel trace), tools/pmc_step.py --parse / --mfma (PMC), the layer report and the JSON lines.
#   bash tools/r5_final.sh tests | bench | pmc | full
case "$1" in
  tests) bash tools/gpu_steps.sh \
    "800 gputests python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
    "120 smoke python -c 'import __graft_entry__ as g; g.smoke()'" ;;
  bench) bash tools/gpu_steps.sh \
    "400 bench python bench.py" \
    "300 btrace env SSSEG_OVERLAP_TEACHER=0 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/btrace -o b -- python bench.py --steps 8 --warmup 3 --no-cpu-baseline --no-fp32 --no-graph" \
    "300 layers python tools/layer_report.py" ;;
  pmc) bash tools/gpu_steps.sh \
    "700 pmc bash tools/pmc_run.sh" \
    "300 full_c5 python tools/full_size_steps.py --configs c5 --graph --train-loop" ;;
  full) bash tools/gpu_steps.sh \
    "900 full_c34 python tools/full_size_steps.py --configs c3,c4 --graph --train-loop" ;;
  *) echo "usage: $0 tests|bench|pmc|full"; exit 2 ;;
esac
