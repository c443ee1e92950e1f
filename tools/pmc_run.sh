set -e
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_f -o f --output-format csv -- python tools/pmc_step.py > gpurun_out/pmc_f.log 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_w -o w --output-format csv -- python tools/pmc_step.py > gpurun_out/pmc_w.log 2>&1
timeout -s KILL 200 rocprofv3 --kernel-trace -d gpurun_out/pmc_t -o t --output-format csv -- python tools/pmc_step.py > gpurun_out/pmc_t.log 2>&1
