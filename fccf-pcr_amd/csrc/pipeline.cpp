// pipeline.cpp — fccf_register: placeholder until the full driver lands.
#include "pipeline.h"
extern "C" int fccf_register(fccf_ctx*, const float*, int64_t, const float*, int64_t, float, const fccf_params*,
                             float*, fccf_stats*) { return FCCF_E_INTERNAL; }
extern "C" int fccf_register_device(fccf_ctx*, const float*, int64_t, const float*, int64_t, float,
                                    const fccf_params*, float*, fccf_stats*) { return FCCF_E_INTERNAL; }
