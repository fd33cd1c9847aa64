set -e
mkdir -p gpurun_out
IZPI_LIB_PATH=$PWD/izpi_amd/_lib/variants/sclk.so timeout -k 10 200 python tools/first_frame.py --config C5 --spp 16 --frames 2 > gpurun_out/c5clk.log 2>&1
grep -a "CLOCKS\|^{\"wall" gpurun_out/c5clk.log
timeout -k 10 200 python tools/first_frame.py --config C5 --spp 16 --frames 3 > gpurun_out/c5new.log 2>&1
grep -a "^{\"wall" gpurun_out/c5new.log
CONFIG=C5 timeout -k 10 400 bash profiles/pmc_kernels.sh c5 8 > gpurun_out/c5pmc.log 2>&1
head -8 gpurun_out/c5pmc.log
