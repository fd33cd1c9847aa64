set -e
timeout -k 10 300 python tools/first_frame.py --config C4 --frames 2 > gpurun_out/ff_ab.log 2>&1
timeout -k 10 300 python tools/first_frame.py --config C4 --frames 2 --slots 48000000 >> gpurun_out/ff_ab.log 2>&1
timeout -k 10 300 python tools/first_frame.py --config C4 --frames 2 --slots 24000000 >> gpurun_out/ff_ab.log 2>&1
timeout -k 10 300 python tools/first_frame.py --config C3 --frames 2 >> gpurun_out/ff_ab.log 2>&1
timeout -k 10 300 python tools/first_frame.py --config C3 --frames 2 --slots 64000000 >> gpurun_out/ff_ab.log 2>&1
timeout -k 10 300 python tools/first_frame.py --config C2 --frames 2 >> gpurun_out/ff_ab.log 2>&1
