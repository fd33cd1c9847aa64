set -e
mkdir -p gpurun_out
for c in "C3 512" "C4 64" "C5 16"; do set -- $c
  for v in tclk sclk; do
    echo "== $1 $v"
    IZPI_LIB_PATH=$PWD/izpi_amd/_lib/variants/$v.so timeout -k 10 200 python tools/first_frame.py --config $1 --spp $2 --frames 2 --stats > gpurun_out/clk_$1_$v.log 2>&1
    grep -E "CLOCKS|^\{\"stats" gpurun_out/clk_$1_$v.log | tail -2
  done
done
