#!/bin/bash
# Final round-3 run of the committed build: the GPU test suite and smoke, then the evidence bundle
# (tools/r3_evidence.sh).  Stops at the first step that faults / times out (tools/gpu_steps.sh).
bash tools/gpu_steps.sh \
  "600 gputests python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread" \
  "120 smoke python -c 'import __graft_entry__ as g; g.smoke()'" && bash tools/r3_evidence.sh
