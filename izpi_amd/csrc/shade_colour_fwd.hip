// shade_colour_fwd.hip — the shading kernels of the Colour sampler, forward (IZPI_ACC_FORWARD) accumulation (shade.h).
#include "shade.h"

template int run_sampler<IZPI_SAMPLER_COLOUR, true>(izpi_ctx*, const izpi_render_req*, const DevScene&, const Tracer&, ShadeParams&,
                                 WaveParams&, AccumParams&, uint32_t, uint32_t, uint32_t, bool, float*, float*, float*,
                                 uint32_t*);
template int prepare_sampler<IZPI_SAMPLER_COLOUR, true>(izpi_ctx*, bool);
