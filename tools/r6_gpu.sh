#!/bin/bash
# Round-6 GPU evidence, in parts that each fit one gpurun call (tools/gpu_steps.sh: every step under its own limit,
# stop at the first fault / time limit).
#   bash tools/r6_gpu.sh tests | full | bench | pmc
case "$1" in
  tests) bash tools/gpu_steps.sh \
    "900 r6_gputests python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider" \
    "120 r6_smoke python -c 'import __graft_entry__ as g; g.smoke()'" ;;
  full) bash tools/gpu_steps.sh \
    "400 r6_full_plain python tools/full_size_steps.py --configs c5,c4 --graph" \
    "400 r6_full_coll python tools/full_size_steps.py --configs c5,c4 --graph --train-loop --collectives" ;;
  bench) bash tools/gpu_steps.sh \
    "400 r6_bench python bench.py" ;;
  quick) bash tools/gpu_steps.sh \
    "600 r6_qtests python -u -m pytest -q --timeout 300 --timeout-method thread -p no:cacheprovider tests/test_c5_fp16.py tests/test_bench_parity.py tests/test_hip_layers.py -k 'oracle or tie_band or ill_conditioned or consumer_dgrad'" ;;
  *) echo "usage: $0 tests|full|bench|quick"; exit 2 ;;
esac
