#!/bin/bash
# Shader clock and power while bench.py runs a long timed region (rocm-smi sampled every 0.5 s), to tell sustained-load
# clocks from the short isolated microbenchmarks'.
#   bash tools/clock_watch.sh gpurun_out/clk
out=${1:-gpurun_out/clk}
mkdir -p "$out"
rocm-smi --showclocks --showpower > "$out/idle.txt" 2>&1
python bench.py --steps 400 --warmup 5 --no-cpu-baseline --no-fp32 > "$out/bench.log" 2>&1 &
pid=$!
for i in $(seq 1 60); do
  if ! kill -0 $pid 2>/dev/null; then break; fi
  echo "=== t=$i" >> "$out/samples.txt"
  rocm-smi --showclocks --showpower >> "$out/samples.txt" 2>&1
  sleep 0.5
done
wait $pid
