/* izpi_gpu_debug.h — test and measurement hooks of libizpi_gpu.so.
 *
 * Not part of the drop-in boundary: the Go shim (integration/go) and INTEGRATION.md's
 * binding do not include this header. The parity tests use the fault injection to drive
 * izpi_gpu_render_rank's failure paths; the workspace re-allocation is the measurement hook
 * behind DESIGN.md section 3.2's placement findings.
 */
#ifndef IZPI_GPU_DEBUG_H
#define IZPI_GPU_DEBUG_H
#include "izpi_gpu.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Fault injection: where = 1 makes izpi_gpu_render_rank fail this rank's local checks, 2
 * makes every render on this context fail as a device fault would, 3 makes this rank's
 * stream stall before the gather as a rank waiting on a dead peer does (released once the
 * call has given up on it), 4 makes izpi_gpu_render_rank's collective waits see a failed
 * stream (a sticky device error): the rank aborts its communicator and returns
 * IZPI_ERR_PEER; 0 = off. */
int izpi_gpu_debug_fault(izpi_ctx* ctx, int where);

/* Re-allocate the render workspace buffers selected by `mask` (bit 0 per-sample results, 1
 * unwinding records, 2 overflow record blocks, 3 their free rings, 4 running sums, 5
 * wavefront state, 6 traversal-stack spill) on other pages: each new buffer is allocated
 * while the old one is still held, then the old one is freed. The contents are not kept
 * (every render rewrites them). */
int izpi_gpu_debug_realloc(izpi_ctx* ctx, uint32_t mask);

#ifdef __cplusplus
}
#endif
#endif
