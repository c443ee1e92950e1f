#!/bin/bash
# A/B of the LDS-DMA placement in the forward/dgrad MFMA stream (knob 11) on the tune-logged bench workload.
bash tools/gpu_steps.sh \
  "300 layertests python -u -m pytest tests/test_hip_layers.py tests/test_vcat.py -x -q --timeout 120 --timeout-method thread" \
  "200 tune_dma0 env SSSEG_TUNE_LOG=1 SSSEG_KNOBS=11=0 python bench.py --steps 20 --no-cpu-baseline --no-fp32" \
  "200 tune_dma1 env SSSEG_TUNE_LOG=1 SSSEG_KNOBS=11=1 python bench.py --steps 20 --no-cpu-baseline --no-fp32" \
  "200 tune_dma2 env SSSEG_TUNE_LOG=1 SSSEG_KNOBS=11=2 python bench.py --steps 20 --no-cpu-baseline --no-fp32"
