# k_trace2 chunk size sweep: A = default build (prefetched queue entries, chunk <= 128),
# B = build without the prefetch, so IZPI_TRACE_CHUNK is not clamped
set -e
cp izpi_amd/_lib/libizpi_gpu.so /tmp/keep.so
cp izpi_amd/_lib/variants/A.so izpi_amd/_lib/libizpi_gpu.so
timeout -k 10 300 python tools/tune.py --spp 512 --rounds 2 --var IZPI_TRACE_CHUNK=64,128 2>&1 | grep VARIANT | sed "s/^/A /"
cp izpi_amd/_lib/variants/B.so izpi_amd/_lib/libizpi_gpu.so
timeout -k 10 400 python tools/tune.py --spp 512 --rounds 2 --var IZPI_TRACE_CHUNK=128,256,512,1024 2>&1 | grep VARIANT | sed "s/^/B /"
cp /tmp/keep.so izpi_amd/_lib/libizpi_gpu.so
