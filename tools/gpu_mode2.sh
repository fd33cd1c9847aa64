# Shading-time modes: clock state inside one process (tools/mode_dpm.py), in a fresh process
# and in one right after a 250-GB hog.
set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/mode_dpm.py > gpurun_out/mode_dpm1.log 2>&1
cat gpurun_out/mode_dpm1.log | grep -v amdgpu.ids
timeout -k 10 120 python -c "import torch; x = torch.empty(int(250e9) // 8, dtype=torch.float64, device='cuda'); x.fill_(1.0); torch.cuda.synchronize(); print('hog 250 GB')"
timeout -k 10 300 python tools/mode_dpm.py > gpurun_out/mode_dpm2.log 2>&1
cat gpurun_out/mode_dpm2.log | grep -v amdgpu.ids
