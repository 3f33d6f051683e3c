// libldm_sdf.so: library-level entry points of the C ABI (include/ldm_sdf.h).
// The compute entry points live next to their kernels (decoder.hip, denoiser.hip).
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>

#include "ldm_internal.h"

namespace ldm {
size_t decoder_workspace_bytes(int B, int dtype, int layout);

static thread_local char g_last_error[512] = "";

void set_error(const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_last_error, sizeof(g_last_error), fmt, ap);
    va_end(ap);
}

#ifdef LDM_DEV_KNOBS
int dev_knob_env(const char* name, int dflt) {
    const char* e = getenv(name);
    return (e && *e) ? atoi(e) : dflt;
}
#endif
}  // namespace ldm

extern "C" int ldm_abi_version(void) { return LDM_ABI_VERSION; }

extern "C" const char* ldm_last_error(void) { return ldm::g_last_error; }

extern "C" size_t ldm_workspace_bytes(int op, int B, int n, int dtype) {
    (void)n;
    if (B < 1) return 0;
    switch (op) {
        case LDM_OP_DECODER_GRID:
        case LDM_OP_DECODER_POINTS:
            return ldm::decoder_workspace_bytes(B, dtype, LDM_LAYOUT_SPLIT);
        default:
            return 0;
    }
}

extern "C" size_t ldm_workspace_bytes_layout(int op, int B, int n, int dtype, int layout) {
    (void)n;
    if (B < 1) return 0;
    switch (op) {
        case LDM_OP_DECODER_GRID:
        case LDM_OP_DECODER_POINTS:
            return ldm::decoder_workspace_bytes(B, dtype, layout);
        default:
            return 0;
    }
}
