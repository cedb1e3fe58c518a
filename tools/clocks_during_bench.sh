#!/bin/bash
# sample the GPU clocks while the bench runs
timeout -k 10 120 python bench.py --steps 400 --warmup 5 --no-cpu-baseline > gpurun_out/clk_bench.json 2> gpurun_out/clk_bench.err &
P=$!
sleep 20
for i in 1 2 3 4 5; do timeout 10 rocm-smi --showclocks --showpower --showtemp 2>/dev/null | grep -i "sclk\|mclk\|fclk\|power\|temp\|edge\|junction" | head -12; sleep 1; done > gpurun_out/clocks.txt
wait $P
cat gpurun_out/clocks.txt | sort | uniq -c | head -30
cut -c1-200 gpurun_out/clk_bench.json
