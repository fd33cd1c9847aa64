# Shading-time modes: C3 at 128 spp in fresh processes, some right after a
# process that filled 250 GB of HBM; each process runs under one rocprofv3 --pmc pass of
# L1->L2 and L2->memory request latency counters and translation counters, so per-process
# k_shade time (the mode) can be set against them.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
set -e
mkdir -p gpurun_out/mode
timeout -s KILL 60 rocprofv3 --list-avail > gpurun_out/mode/avail_all.txt 2>&1 || true
grep -o -E "\b(TCP_TCC_[A-Z_]*LATENCY[A-Z_]*|TCP_TCC_READ_REQ|TCP_TCC_WRITE_REQ|TCC_EA0?_RDREQ_LEVEL|TCC_EA0?_WRREQ_LEVEL|TCC_EA0?_RDREQ|TCC_EA0?_WRREQ|TCP_UTCL1_[A-Z_]*|UTCL2[A-Z_]*|TCC_[A-Z_]*LATENCY[A-Z_]*)\b" gpurun_out/mode/avail_all.txt | sort -u > gpurun_out/mode/avail.txt || true
cat gpurun_out/mode/avail.txt
pick() { for c in "$@"; do if grep -qx "$c" gpurun_out/mode/avail.txt; then printf "%s_sum " "$c"; fi; done; }
A="$(pick TCP_TCC_READ_REQ_LATENCY TCP_TCC_WRITE_REQ_LATENCY TCP_TCC_READ_REQ TCP_TCC_WRITE_REQ)$(pick TCC_EA0_RDREQ_LEVEL TCC_EA0_RDREQ TCC_EA0_WRREQ_LEVEL TCC_EA0_WRREQ)"
B="$(pick TCP_UTCL1_TRANSLATION_MISS TCP_UTCL1_TRANSLATION_HIT TCP_UTCL1_PERMISSION_MISS TCP_UTCL1_REQUEST)"
echo "A: $A"; echo "B: $B"
hog() { timeout -k 10 120 python -c "import torch; x = torch.empty(int(250e9) // 8, dtype=torch.float64, device='cuda'); x.fill_(1.0); torch.cuda.synchronize(); print('hog 250 GB')"; }
run() {  # tag counters
  timeout -s KILL 150 rocprofv3 --pmc $2 --kernel-trace --output-format csv -d gpurun_out/mode/$1 -o run -- python3 tools/first_frame.py --config C3 --frames 2 --spp 128 > gpurun_out/mode/$1.log 2>&1 || { echo "pass $1 failed"; tail -5 gpurun_out/mode/$1.log; exit 1; }
  grep '^{"config' gpurun_out/mode/$1.log | tail -1 | cut -c1-400
}
run a1 "$A"
run b1 "$B"
hog
run a2 "$A"
hog
run b2 "$B"
run a3 "$A"
hog
run a4 "$A"
run b3 "$B"
hog
run b4 "$B"
